# SQ instruction-mix counters of the chain kernel (config 3, one store, run8)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
SETTINGS=${SETTINGS:-run8} STEPS=3 timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/tools/chain_sweep.py > $R/gpurun_out/pmc_sq.log 2>&1
rc=$?; echo "sq rc=$rc"; tail -3 $R/gpurun_out/pmc_sq.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
SETTINGS=${SETTINGS:-run8} STEPS=3 timeout -s KILL 400 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_sq2 -o run -- python3 $R/tools/chain_sweep.py > $R/gpurun_out/pmc_sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; tail -3 $R/gpurun_out/pmc_sq2.log | cut -c1-300
exit $rc
