# Round-5 close on the final library: thin-wgrad bitwise check vs the previous build, full GPU suite, smoke, profile
set -o pipefail
mkdir -p gpurun_out/r5e
VQA_LIB_PATH=variants/old.so timeout -k 10 120 python tools/thin_time.py --save gpurun_out/r5e/old.pt 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/thin_time.py --check gpurun_out/r5e/old.pt 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r5e/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r5e/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5e/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1 || exit 1
rm -f variants/old.so
bash tools/round_profile.sh r5e || exit 1
