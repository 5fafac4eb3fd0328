cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && timeout -k 10 200 python3 tools/config5_probe.py 20 > gpurun_out/c5.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/c5.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_config5_trace.sh
