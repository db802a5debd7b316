# the request pass's PMC traffic (FETCH_SIZE, WRITE_SIZE: separate runs,
# kernel trace only) on 4 rotating 1 M batches in the bench step's output
# form, folded into traffic_genome.json (copy it to profiles/ for bench.py)
TAG=${TAG:-gpu_pass_traffic}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
step save 300 python3 -u $R/tools/req_tune.py --save /tmp/st --rounds 3 --digest
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o p -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 2
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o p -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 2
step traffic 60 python3 $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write --out $O/traffic_genome.json --records 85000000 --requests 1000000 --kernel request_eval_kernel --batches 4
exit 0
