"""Isolated range-proof passes of several sizes: wall ms per pass, verifies/s and
per-kernel device times (A/B of the com paths via FTS_COM_FIXED_MAX).
    python tools/pass_times.py 4096 16384 32768"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
import fts_gpu  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [4096]
raw = open(os.path.join(ROOT, "tests/golden/zkatdlog_pp.json"), "rb").read()
pp = fts_gpu.PublicParams(raw, bit_length=64, device=0)
rng = random.Random(5)
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
base = 4096
vals = [rng.getrandbits(64) for _ in range(base)]
bfs = [rng.randrange(R).to_bytes(32, "big") for _ in range(base)]
proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=9)
tag = os.environ.get("TAG", "")
for B in sizes:
    m = B // base
    b = pp.stage_range_proofs(proofs * m, coms * m)
    reps, acc, t = 5, {}, 0.0
    for r in range(reps + 1):
        t0 = time.perf_counter()
        st = b.verify()
        dt = time.perf_counter() - t0
        assert int((st != 0).sum()) == 0
        if r:
            t += dt / reps
            for k, (ms, mads) in b.timings().items():
                acc[k] = acc.get(k, 0.0) + ms / reps
    print("%s B=%d wall=%.3f ms (%.2f M/s) " % (tag, B, t * 1e3, B / t / 1e6)
          + " ".join("%s=%.3f" % (k, v) for k, v in acc.items() if not k.startswith("host_") or k == "host_wait_flag"),
          flush=True)
    b.close()
