set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ac; mkdir -p $O
T="timeout -k 10"
for v in 16384 49152 16384 49152 16384 49152; do
  FTS_COM_FIXED_MAX=$v $T 240 python3 -u tools/burst.py --steps 20 --reps 9 --tag cfm$v >> $O/burst.log 2>&1 || exit 1
done
echo rc=$?
