#!/bin/bash
# Round-3 GPU session steps (run on the box through gpurun from the repo root).
#   tools/gpu_r03.sh tests      full -m gpu suite
#   tools/gpu_r03.sh identity   identity bench on both curves + rocprofv3 kernel stats
#   tools/gpu_r03.sh rp         C2 headline (driver shape and 512 steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03
mkdir -p $O
case "$1" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
    rc=$?; tail -3 $O/pytest_gpu.log; exit $rc ;;
  identity)
    for c in bn254 fp256bn; do
      timeout -k 10 300 python bench.py --workload identity --idemix-curve $c --steps 10 --warmup 2 \
        > $O/bench_identity_$c.json 2> $O/bench_identity_$c.err || exit $?
    done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/prof_identity -o prof -- \
      python3 bench.py --workload identity --steps 4 --warmup 1 --cpu-sample 0 > $O/prof_identity.log 2>&1 ;;
  rp)
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err &&
    timeout -k 10 300 python bench.py --cpu-sample 0 > $O/bench_s512.json 2> $O/bench_s512.err ;;
  *) echo "usage: $0 tests|identity|rp"; exit 2 ;;
esac
