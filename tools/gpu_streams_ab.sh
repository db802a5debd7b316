# The config-3 rotation with independent batches on 1, 2 or 4 streams
# (tools/req_tune.py --streams): does overlapping consecutive batches' passes
# raise the step rate?  Digests must equal.  Outputs under gpurun_out/$TAG.
TAG=${TAG:-streams}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -n 1 $O/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step save 400 python3 -u $R/tools/req_tune.py --save /tmp/st --rounds 2 --digest
i=0
for n in ${NS:-2 4 2 4}; do
  i=$((i+1))
  step s${i}_$n 200 python3 -u $R/tools/req_tune.py --open /tmp/st --rounds ${ROUNDS:-15} --streams $n --digest
done
exit 0
