timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_head.py -m gpu -p no:cacheprovider > gpurun_out/head_tests.log 2>&1; tail -3 gpurun_out/head_tests.log; grep -E "^E |FAILED" gpurun_out/head_tests.log | head -20
TAG=b ALTS="prio2 skewA skewB skewAa main" bash scripts/r6/bip_alt.sh
