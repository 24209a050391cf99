#!/bin/bash
# GPU job runner for gpurun: each GPU step under its own timeout; stop at the
# first fault / abort / timeout (exit 124, 134, 137, 139). Test failures (exit 1)
# do not stop later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  case $rc in 0|1|5) return 0 ;; *) echo "STOP after $name (rc=$rc)"; exit $rc ;; esac
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    alltests) step pytest_all 1200 python -m pytest tests -q -x ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchq) step bench 300 python bench.py --steps 20 --no-cpu ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 20 --no-cpu --no-plan ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
