set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04i; mkdir -p $O
T="timeout -k 10"
for lib in fabric-token-sdk_amd/lib/libfts_gpu.so fabric-token-sdk_amd/lib/ab/join_in.so fabric-token-sdk_amd/lib/libfts_gpu.so fabric-token-sdk_amd/lib/ab/join_in.so; do
  FTS_LIB=$lib $T 200 python3 -u tools/pass_times.py 81920 >> $O/pass.log 2>&1 || exit 1
  FTS_LIB=$lib $T 200 python3 -u tools/burst.py --steps 20 --reps 9 --tag $(basename $lib) >> $O/burst.log 2>&1 || exit 1
done
FTS_LIB=fabric-token-sdk_amd/lib/ab/join_in.so $T 300 python3 -u tools/burst.py --steps 512 --reps 2 --tag join512 >> $O/burst.log 2>&1
echo rc=$?
