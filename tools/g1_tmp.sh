set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04y; mkdir -p $O
T="timeout -k 10"
for i in 0 1 0 1 0 1; do
  echo "shape=$i" >> $O/s20.txt
  $T 200 python3 -u bench.py --steps 20 --warmup 5 --shape-warmup $i --host-steps 0 --cpu-sample 0 >> $O/s20.txt 2>> $O/s20.err || exit 1
done
echo rc=$?
