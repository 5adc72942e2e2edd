# round-4 producer / pipeline A/B: Gram + C2 tests, the in-line flow against the
# previous commit's library, the pipelined flow with and without CU masks, and
# a kernel timeline of the pipelined flow
set -o pipefail
O=gpurun_out
TAG=${TAG:-r04n}
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_configs.py -k "gram or xw or cu_mask or c2_fast or localsgd" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1 || { tail -30 $O/tests_$TAG.log; exit 1; }
tail -1 $O/tests_$TAG.log
VARIANTS="base prev" TAG=$TAG tools/gpu_run.sh ab || exit $?
BENCH_ARGS="--pipeline" VARIANTS="base base+COCOA_CU_MASK=1 base+COCOA_EVAL_ON_GSTREAM=1" TAG=${TAG}_pipe tools/gpu_run.sh ab || exit $?
COCOA_CU_MASK=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_pipe_$TAG -o run --output-format csv -- python3 bench.py --pipeline --steps 6 --warmup 2 --no-cpu-baseline --no-gap > $O/tl_pipe_$TAG.log 2>&1 || exit $?
python3 tools/timeline.py $O/tl_pipe_$TAG 2 > $O/tl_pipe_$TAG.txt || exit $?
cat $O/tl_pipe_$TAG.txt
