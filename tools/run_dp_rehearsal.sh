#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: 2 ranks sharing cuda:0 over gloo (the
# driver's 8-GPU runs use RCCL; this checks the sharding, barriers, max-over-ranks timing,
# parameter broadcast and the summed point count).  Small grid to keep both ranks in memory.
mkdir -p gpurun_out
export PCS_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --grid 64 --no-cpu-baseline --no-kernel-timing \
  > gpurun_out/dp_rehearsal.json 2> gpurun_out/dp_rehearsal.err
rc=$?
cat gpurun_out/dp_rehearsal.json; tail -5 gpurun_out/dp_rehearsal.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --workload cfg3 --occupancy 0.002 --no-cpu-baseline \
  --no-kernel-timing > gpurun_out/dp_rehearsal_cfg3.json 2>> gpurun_out/dp_rehearsal.err
rc=$?
cat gpurun_out/dp_rehearsal_cfg3.json
exit $rc
