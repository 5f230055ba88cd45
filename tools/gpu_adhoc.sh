# ad-hoc GPU step: identity pairing with inlined Fp6 products (A/B library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03j; mkdir -p $O
AB=fabric-token-sdk_amd/lib/ab/idv_inl.so
FTS_LIB=$AB timeout -k 10 400 python3 -u -m pytest tests/test_idemix_identity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for L in fabric-token-sdk_amd/lib/libfts_gpu.so $AB; do for c in bn254 fp256bn; do
  FTS_LIB=$L timeout -k 10 200 python3 bench.py --workload identity --idemix-curve $c --steps 12 --warmup 2 --cpu-sample 0 > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
  grep '^{' $O/b.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$L $c', d['value'], d['kernel_ms'])"
done; done
