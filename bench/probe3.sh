# r3 irregular-SpMV probes (bench/gather_probe.hip): paced tile kernel + L2 counters
cd $GRAFT_REPO_ROOT
timeout -k 10 240 ./build/gather_probe tiles > gpurun_out/r3_gather_probe4.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in 8; do
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r3_pmc_tile_p$P -o pmc --output-format csv -- ./build/gather_probe tile 262144 1024 0 $P > gpurun_out/r3_pmc_tile_p$P.txt 2>&1 || exit 1
done
