export TMPDIR=/tmp
so=lz4-sgori_amd/lz4e_amd/liblz4e_amd.so
for v in lz4-sgori_amd/build/var/lib*.so; do
  cp $v $so
  rm -rf gpurun_out/wt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/wt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong > gpurun_out/wt.log 2>&1
  echo "== $v"; grep -E "weight_kernel|compress_kernel" $(find gpurun_out/wt -name "*kernel_stats.csv" | head -1) | cut -c1-80
done
