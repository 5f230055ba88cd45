"""Where the time of one fts_transfer_verify_batch call goes (host vs device):
python tools/transfer_profile.py [n_transfers]"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402

import fts_gpu  # noqa: E402
from fts_gpu import _lib as L  # noqa: E402

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
pp = fts_gpu.PublicParams(open(os.path.join(ROOT, "tests/golden/zkatdlog_pp.json"), "rb").read(), bit_length=64)
rng = random.Random(4)
base = []
for i in range(256):
    a, b = rng.getrandbits(62), rng.getrandbits(62)
    c = rng.randrange(a + b + 1)
    ib = [rng.randrange(R).to_bytes(32, "big") for _ in range(2)]
    ob = [rng.randrange(R).to_bytes(32, "big") for _ in range(2)]
    ins = [pp.token_commit(b"ABC", v, x) for v, x in zip([a, b], ib)]
    outs = [pp.token_commit(b"ABC", v, x) for v, x in zip([c, a + b - c], ob)]
    base.append((ins, outs, pp.prove_transfer(b"ABC", [a, b], ib, [c, a + b - c], ob, i)))
items = [base[i % 256] for i in range(n)]
pp.verify_transfers(items)
t0 = time.perf_counter()
arr = (L.TransferItem * n)()
keep = []
for i, (ins, outs, proof) in enumerate(items):
    bi = C.create_string_buffer(b"".join(ins))
    bo = C.create_string_buffer(b"".join(outs))
    bp = C.create_string_buffer(proof, len(proof))
    keep += [bi, bo, bp]
    arr[i] = L.TransferItem(C.cast(bi, C.c_void_p), 2, C.cast(bo, C.c_void_p), 2, C.cast(bp, C.c_void_p), len(proof))
t1 = time.perf_counter()
st = np.zeros(n, dtype=np.int32)
fi = np.zeros(n, dtype=np.int32)
for _ in range(3):
    t2 = time.perf_counter()
    L.lib.fts_transfer_verify_batch(pp._ctx, n, arr, st.ctypes.data_as(C.POINTER(C.c_int32)),
                                    fi.ctypes.data_as(C.POINTER(C.c_int32)))
    t3 = time.perf_counter()
tm = pp.last_timings_ex()
dev = sum(v[0] for k, v in tm.items() if k == "host_wait_flag")
print("python item build %.1f ms, C call %.1f ms, host_prep %.2f enqueue %.2f wait_flag %.2f, sig %.2f, ok=%d" % (
    (t1 - t0) * 1e3, (t3 - t2) * 1e3, tm.get("host_prep", (0,))[0], tm.get("host_enqueue", (0,))[0],
    tm.get("host_wait_flag", (0,))[0], tm.get("k_sig_finish", (0,))[0], int((st == 0).sum())))
print("host:", {k: round(v[0], 3) for k, v in tm.items() if k.startswith("host_")})
print("kernels:", {k: round(v[0], 3) for k, v in tm.items() if not k.startswith("host_")})
