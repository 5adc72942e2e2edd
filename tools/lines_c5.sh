cd ${GRAFT_REPO_ROOT}
O=gpurun_out
for m in cocoa mbcd mbsgd localsgd; do
  timeout -k 10 300 python3 bench.py --method $m --steps 10 --warmup 2 --cpu-seconds 8 > $O/line_c5_${m}_r07w.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.loads(open('$O/line_c5_${m}_r07w.json').readlines()[-1]);print('$m', round(d['ms_per_step'],3), round(d['value']/1e6,1), {k: round(v,3) for k,v in d['kernel_ms'].items()})"
done
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gap > $O/line_c2_r07w.json 2>/dev/null && python3 -c "import json;d=json.loads(open('$O/line_c2_r07w.json').readlines()[-1]);print('c2', round(d['ms_per_step'],3))"
