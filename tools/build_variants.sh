#!/bin/bash
# Builds libpcs.so variants of one source (SRC, default gemm_glds) with extra -D flags into
# abtest/<name>/libpcs.so:
#   [SRC=small] tools/build_variants.sh name1 "-DX=1" name2 "-DY=1 -DZ=1" ...
set -e
cd "$(dirname "$0")/.."
C=point-cloud-cnn-segmentation_amd/csrc
SRC=${SRC:-gemm_glds}
make -C $C -j8 >/dev/null
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p abtest/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -disable-machine-sink $flags \
    -c $C/$SRC.hip -o abtest/$name/$SRC.o
  objs=$(ls $C/*.o | grep -v "/$SRC.o")
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o abtest/$name/libpcs.so abtest/$name/$SRC.o $objs
done
