# round 6: entropy encoder phase stamps (diag build) + kernel-time A/B of variants
#   bash tools/r06_t.sh "<diag names>" "<ab libs>"
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
for n in $1; do
  timeout -k 10 200 python -u tools/ent_ephase.py $n > $O/ephase_$n.log 2>&1 || { cat $O/ephase_$n.log; exit 1; }
  cat $O/ephase_$n.log
done
if [ -n "$2" ]; then
  timeout -k 10 300 python -u tools/ab_ent_inproc.py 40 $2 > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; exit $rc
fi
