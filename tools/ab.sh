#!/bin/bash
# tools/ab.sh NAME ROUNDS TIMEOUT CMD VARIANT... — interleaved A/B of library builds
# and / or environment settings on one GPU box (diagnostic tool).
#   VARIANT: comma-separated items, each lib=PATH (run against that build through
#            RBE_LIB_PATH) or KEY=VALUE (an environment setting); "-" = as is.
#   CMD:     one shell command, run once per variant and round under
#            timeout -k 10 TIMEOUT; its output is appended to gpurun_out/ab_NAME.log
#            below a "== round R: VARIANT" header. Stops at the first failing run.
# Examples (the round-4 one-off scripts that profiles/r04 cites, as invocations):
#   ab_conn.sh:  tools/ab.sh conn 2 300 "python tools/well_ab.py dense=RBE_EDGE_PACKED:0" \
#                    RBE_EDGE_CONN_ROUNDS=0 RBE_EDGE_CONN_ROUNDS=4 RBE_EDGE_CONN_ROUNDS=8
#   ab_seeds.sh: tools/ab.sh seeds 2 300 "python tools/well_ab.py dense=RBE_EDGE_PACKED:0" \
#                    - lib=abvariants/lib_s32.so lib=abvariants/lib_s128.so
#   ab_edges*.sh, ab_g5.sh: tools/ab.sh edges 2 200 "rocprofv3 --kernel-trace --stats --output-format csv \
#                    -d gpurun_out/eab -o kt -- python tools/edge_bench.py --scene clutter64" - lib=abvariants/lib_ew5.so
#   ab_spec.sh, ab_ml.sh, ab_fm.sh, ab_mledge.sh, ab_qpad.sh: the same with their
#                    abvariants builds against tools/well_ab.py / tools/plan_bench.py
set -o pipefail
[ $# -ge 5 ] || { sed -n 2,20p "$0"; exit 2; }
name=$1 rounds=$2 tmo=$3 cmd=$4
shift 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
log=gpurun_out/ab_$name.log
: > "$log"
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    echo "== round $r: $v" >> "$log"
    envs=()
    if [ "$v" != "-" ]; then
      IFS=',' read -ra items <<< "$v"
      for it in "${items[@]}"; do
        case $it in
          lib=*) envs+=("RBE_LIB_PATH=${it#lib=}") ;;
          *=*) envs+=("$it") ;;
          *) echo "bad variant item $it" >&2; exit 2 ;;
        esac
      done
    fi
    env "${envs[@]}" timeout -k 10 "$tmo" bash -c "$cmd" 2>&1 | grep -v amdgpu.ids >> "$log" || { echo "FAILED: $v" >> "$log"; exit 1; }
  done
done
echo "ab $name done: $log"
