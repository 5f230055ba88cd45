"""Driver-shaped bursts of the C2 headline: K batch verifications of 4,096 rp64
proofs submitted at once from K host threads (bench.py --steps K), repeated
--reps times in one process; prints the median rate and the per-burst rates.
Library knobs (FTS_LANES, FTS_COALESCE_MAX, FTS_GATHER_US, ...) come from the
environment, so an A/B is one process per setting.
    python tools/burst.py --steps 20 --reps 7"""
import argparse
import json
import os

# as bench.py: 16 hardware queues (read once when HIP loads)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=7)
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--tag", default="")
a = ap.parse_args()
import fts_gpu  # noqa: E402

pp = fts_gpu.PublicParams(open(os.path.join(ROOT, "tests/golden/zkatdlog_pp.json"), "rb").read(), bit_length=64, device=0)
pp.reserve()
rng = random.Random(3)
vals = [rng.getrandbits(64) for _ in range(a.batch)]
bfs = [rng.randrange(R).to_bytes(32, "big") for _ in range(a.batch)]
proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=11)
batches = [pp.stage_range_proofs(proofs, coms) for _ in range(a.steps)]


def burst():
    out = [None] * a.steps

    def run(i):
        out[i] = (batches[i].verify(want_status=True), batches[i].merged())
    gate = threading.Barrier(a.steps + 1)  # as bench.py: submitters released together

    def body(i):
        gate.wait()
        run(i)
    th = [threading.Thread(target=body, args=(i,)) for i in range(a.steps)]
    for t in th:
        t.start()
    t0 = time.perf_counter()
    gate.wait()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    assert all(int((st != 0).sum()) == 0 for st, _ in out)
    return dt, sum(m for _, m in out) / a.steps


burst()
burst()
res = [burst() for _ in range(a.reps)]
rates = sorted(a.steps * a.batch / dt for dt, _ in res)
print(json.dumps({"tag": a.tag, "steps": a.steps, "median": round(rates[len(rates) // 2]), "min": round(rates[0]),
                  "max": round(rates[-1]), "merged": round(sum(m for _, m in res) / len(res), 2),
                  "env": {k: v for k, v in os.environ.items() if k.startswith("FTS_")}}))
