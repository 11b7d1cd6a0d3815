# seg4 timing ablations: abtest/a<N>/libpcs.so built with -DSEG4_ABL=N (wrong results, timing only)
for v in base $(ls abtest); do
  if [ $v = base ]; then L=point-cloud-cnn-segmentation_amd/csrc/libpcs.so; else L=abtest/$v/libpcs.so; fi
  echo "== $v"; PCS_LIB=$L timeout -k 10 120 python tools/bench_seg.py 5 2>&1 | grep -v amdgpu.ids || exit 1
done
