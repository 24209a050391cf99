# connect launches: loop-free k_edges over each group's first R rounds, then one wave
# per group for the rest (RBE_EDGE_CONN_ROUNDS = R; 0: every round loop-free): C5
# covered-well plans (tools/well_ab.py, same plans), two interleaved rounds
set -o pipefail
rm -f gpurun_out/ab_conn.log
for r in 1 2; do
  for v in 0 4 8; do
    echo "== RBE_EDGE_CONN_ROUNDS=$v" >> gpurun_out/ab_conn.log
    RBE_EDGE_CONN_ROUNDS=$v timeout -k 10 300 python tools/well_ab.py dense=RBE_EDGE_PACKED:0 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_conn.log || exit 1
  done
done
