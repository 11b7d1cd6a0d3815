#!/bin/bash
# Builds timing-ablation variants of libpcs.so (gemm_glds.hip compiled with -DPCS_ABL=v) into
# abtest/abl<v>/libpcs.so; run a variant with PCS_LIB=abtest/abl<v>/libpcs.so.
set -e
cd "$(dirname "$0")/.."
C=point-cloud-cnn-segmentation_amd/csrc
make -C $C -j8 >/dev/null
for v in "$@"; do
  mkdir -p abtest/abl$v
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -disable-machine-sink -DPCS_ABL=$v \
    -c $C/gemm_glds.hip -o abtest/abl$v/gemm_glds.o
  objs=$(ls $C/*.o | grep -v gemm_glds.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o abtest/abl$v/libpcs.so abtest/abl$v/gemm_glds.o $objs
done
