mkdir -p gpurun_out
timeout -k 10 300 python -u tools/decab.py 256 > gpurun_out/decab.txt 2>&1; rc=$?; cat gpurun_out/decab.txt; exit $rc
