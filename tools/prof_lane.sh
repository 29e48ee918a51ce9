cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proflane -o run -- python3 tools/decmodes.py ${MODES:-7} ${WL:-sil4k,fio4k} > gpurun_out/proflane.log 2>&1 || { tail -20 gpurun_out/proflane.log; exit 1; }
grep "==" gpurun_out/proflane.log
python3 tools/rocpd_stats.py $(find gpurun_out/proflane -name "*.db" | head -1) | head -12
