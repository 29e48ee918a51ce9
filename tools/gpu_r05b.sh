#!/bin/bash
# Round 5: the band compressor on the GPU: compress parity tests, every frame
# of the full-size configs, then the default bench (band vs wave compressor).
tag=${1:-r05b}
o=gpurun_out/$tag; mkdir -p $o
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 3 "$o/$name.log" | cut -c1-1500 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
step pytest_c 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compress_batch or byu64 or limited or kat or edge or sg_batch or launch_order"
step pytest_full 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "full_size_every_frame or sg512_layout"
B=(--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-single-call --no-strong)
step bench_band 300 python -u bench.py "${B[@]}"
LZ4E_COMPRESS_MODE=wave step bench_wave 300 python -u bench.py "${B[@]}"
step bench_t256 300 python -u bench.py --workload text256k "${B[@]}"
