timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/trim_tests.log 2>&1 || { tail -30 gpurun_out/trim_tests.log; exit 1; }
tail -1 gpurun_out/trim_tests.log
VARIANTS="base=abl/lib_base.so trim=abl/lib_trim.so" bash tools/gpu_ab3.sh
