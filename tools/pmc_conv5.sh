# PMC passes over tools/bench_conv5.py (the conv5 BN+ReLU pass kernels), one pass per counter
# group, each under its own time limit
set -e
mkdir -p gpurun_out/pmc_c5
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_c5/avail.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_c5/sq1 -o run -- python3 tools/bench_conv5.py > gpurun_out/pmc_c5/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_c5/sq2 -o run -- python3 tools/bench_conv5.py > gpurun_out/pmc_c5/sq2.log 2>&1
