# r3: tiles segment sweep + co-run probe with register-pressure controls under a kernel trace
cd $GRAFT_REPO_ROOT
S="--problem randspd --rows 100000000 --band 410 --density 1.0 --scramble 1 --sim-world 8 --sim-rank 3 --steps 6 --warmup 2 --phases 0 --no-verify"
for cfg in "tile_seg_log2=20" "tile_seg_log2=21" "tile_seg_log2=22" "tile_pace=2,tile_seg_log2=20" "tile_pace=2,tile_seg_log2=21"; do
  sets=""; for kv in ${cfg//,/ }; do sets="$sets --set $kv"; done
  timeout -k 10 300 python bench.py $S $sets > gpurun_out/r3_tsweep_${cfg//[=,]/_}.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/r3_tsweep_${cfg//[=,]/_}.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'])"
done
timeout -k 10 240 python bench/corun_probe.py --reps 4 > gpurun_out/r3_corun.json 2> gpurun_out/r3_corun.err || { tail -5 gpurun_out/r3_corun.err; exit 1; }
cat gpurun_out/r3_corun.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3_corun_trace -o corun --output-format csv -- python3 bench/corun_probe.py --reps 2 > gpurun_out/r3_corun_traced.json 2> gpurun_out/r3_corun_traced.err || { tail -5 gpurun_out/r3_corun_traced.err; exit 1; }
f=$(find gpurun_out/r3_corun_trace -name "*kernel_trace.csv" | head -1)
python bench/corun_trace.py $f > gpurun_out/r3_corun_trace_summary.txt && head -40 gpurun_out/r3_corun_trace_summary.txt
