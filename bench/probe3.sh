# r3 irregular-SpMV probes (bench/gather_probe.hip): L2 counters of the bisection variants
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for F in 0 1 4 8; do
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d gpurun_out/r3_pmc_tt$F -o pmc --output-format csv -- ./build/gather_probe tt $F > gpurun_out/r3_pmc_tt$F.txt 2>&1 || exit 1
done
