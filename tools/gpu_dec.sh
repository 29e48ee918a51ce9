mkdir -p gpurun_out
timeout -k 10 300 python -u tools/decab.py 256 > gpurun_out/decab.txt 2>&1; rc=$?; cat gpurun_out/decab.txt; [ $rc -ne 0 ] && exit $rc
LZ4E_PIPE_OCC5=1 timeout -k 10 300 python -u tools/decab.py 256 > gpurun_out/decab5.txt 2>&1; rc=$?; echo "=== occ5"; grep "==" gpurun_out/decab5.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "decompress or full_size or chunk" > gpurun_out/pytest_dec.log 2>&1; rc=$?
tail -n 5 gpurun_out/pytest_dec.log
exit $rc
