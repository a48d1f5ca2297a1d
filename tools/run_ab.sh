set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
BDLS_HIP_LIB=$PWD/exp/libbdlship_t8.so BH_LL_T=8 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_t8.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_t8.log; [ $rc -le 1 ] || exit $rc
for pass in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --side-configs 0 > gpurun_out/exp_t7_p$pass.json 2> gpurun_out/exp_t7_p$pass.err || exit $?
  BDLS_HIP_LIB=$PWD/exp/libbdlship_t8.so BH_LL_T=8 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --side-configs 0 > gpurun_out/exp_t8_p$pass.json 2> gpurun_out/exp_t8_p$pass.err || exit $?
done
echo DONE
