set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06f/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r06f/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r06f/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06f/smoke.log 2>&1 || { tail -20 gpurun_out/r06f/smoke.log; exit 1; }
tail -1 gpurun_out/r06f/smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r06f/bench.json 2> gpurun_out/r06f/bench.err || { tail -20 gpurun_out/r06f/bench.err; exit 1; }
cat gpurun_out/r06f/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().split(chr(10))[-1]); print(d['value'], d['ms_per_step'], d.get('roofline'), d.get('single_call'), d.get('strong',{}).get('block_floor'))"
