# r3: tiles pacing / segment-size sweep at the scrambled config-5 P = 8 share (profiles/r3_config5_scrambled.md)
cd $GRAFT_REPO_ROOT
S="--problem randspd --rows 100000000 --band 410 --density 1.0 --scramble 1 --sim-world 8 --sim-rank 3 --steps 6 --warmup 2 --phases 0 --no-verify"
for cfg in "tile_pace=1" "tile_pace=2" "tile_pace=0" "tile_seg_log2=17" "tile_seg_log2=19" "tile_pace=2,tile_seg_log2=19"; do
  sets=""; for kv in ${cfg//,/ }; do sets="$sets --set $kv"; done
  timeout -k 10 300 python bench.py $S $sets > gpurun_out/r3_tsweep_${cfg//[=,]/_}.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/r3_tsweep_${cfg//[=,]/_}.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'])"
done
