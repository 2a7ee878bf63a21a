# round 6: where and when the entropy decode waves run (diag build)
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 200 python -u tools/ent_diag.py > $O/diag.log 2>&1; rc=$?; cat $O/diag.log; exit $rc
