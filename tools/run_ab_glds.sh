for L in point-cloud-cnn-segmentation_amd/csrc/libpcs.so gpurun_libs/libpcs_NOEXTRACT.so gpurun_libs/libpcs_NOSELECT.so gpurun_libs/libpcs_NOS1.so; do
  echo "== $L"; PCS_LIB=$L timeout -k 10 200 python tools/bench_glds.py 2>/dev/null | grep "dgrad: mask + store  " || exit 1
done
