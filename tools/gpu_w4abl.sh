# w4 timing ablations (tools/bench_w4.py with W4_ONLY, one alternative build per W4_ABL value)
set -o pipefail
mkdir -p gpurun_out
D=point-cloud-cnn-segmentation_amd/csrc/abl
for n in ${ABL_LIST:-6 22 38 54 102 230}; do
  echo "== W4_ABL=$n"
  PCS_LIB=$D/libpcs_w4abl$n.so W4_ONLY=1 timeout -k 10 120 python -u tools/bench_w4.py || exit $?
done 2>&1 | tee gpurun_out/w4_abl.log
