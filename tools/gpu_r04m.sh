set -o pipefail
VARIANTS="base prev gv1 base prev" TAG=r04m tools/gpu_run.sh ab || exit $?
O=gpurun_out
for m in pipe inline; do
  a=""; [ $m = pipe ] && a="--pipeline"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_${m}_r04m -o run --output-format csv -- python3 bench.py $a --steps 6 --warmup 2 --no-cpu-baseline --no-gap > $O/tl_${m}_r04m.log 2>&1 || exit $?
  python3 tools/timeline.py $O/tl_${m}_r04m 2 > $O/tl_${m}_r04m.txt || exit $?
done
cat $O/tl_pipe_r04m.txt | head -60
