# round-end validation and evidence (round 6): smoke, every GPU test, the
# default bench line (config 3, with its config-4 sub-object: bench_paths at
# 50 datasets), a
# rocprofv3 kernel summary of the default bench, and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE: separate runs, kernel trace only) of the rotating
# config-3 request passes folded into traffic_genome.json; stops at the
# first failure.  Outputs under gpurun_out/$TAG (default final).
TAG=${TAG:-final}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
# PARTS: which of tests / bench / prof / pmc to run (default all; one
# gpurun call holds at most 1,200 s, so the final evidence is two calls)
has() { case " ${PARTS:-tests bench prof pmc} " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
fi
has bench && step bench 600 python3 -u $R/bench.py --steps 20 --warmup 5
cd /tmp
has prof && step prof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline
has pmc || exit 0
step save 300 python3 -u $R/tools/req_tune.py --save /tmp/st --rounds 3 --digest
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o p -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 2
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o p -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 2
step traffic 60 python3 $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write --out $O/traffic_genome.json --records 85000000 --requests 1000000 --kernel request_eval_kernel --batches 4
exit 0
