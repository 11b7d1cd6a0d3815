set -e
export TMPDIR=/tmp
O=gpurun_out/pmc_cal
mkdir -p $O
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 tools/pmc_calibrate.py > $O/f.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 tools/pmc_calibrate.py > $O/w.log 2>&1
