set -e
export TMPDIR=/tmp
O=gpurun_out/pmc_big
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 tools/prof_big.py fwd 2 > $O/p1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/p2 -o run -- python3 tools/prof_big.py fwd 2 > $O/p2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p3 -o run -- python3 tools/prof_big.py fwd 2 > $O/p3.log 2>&1
