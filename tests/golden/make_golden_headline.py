"""Golden fixtures at the headline shapes (BASELINE configs C1/C4 and C5):
64-bit 2-in/2-out transfers and issues with 16 outputs at 32 bits, made by the
CPU oracle (oracle/zkat.py, the restatement of the reference provers and
verifiers).

Cases (reference tests they follow):
  transfers, 64-bit  transfer/transfer_test.go:49-84,130-184 (honest, wrong sum,
                     out of range), typeandsum_test.go:87-142 (wrong type, wrong
                     values, wrong blinding factors), plus tampered T1 / L_j /
                     Delta inside the RangeCorrectness proof (bulletproof.go:314-323,
                     ipa.go:258 error classes at a given index)
  issues, 32-bit x16 issue/issue_test.go:15-22 (honest), a token committed to
                     another value (range failure at its index), a tampered
                     SameType challenge (sametype.go:180)

    python tests/golden/make_golden_headline.py      # rewrites headline_golden.json (~2 min, 8 processes)
"""
import json
import os
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bn254 as bn, der, pp as ppm, zkat  # noqa: E402

T = b"ABC"


def pt(p):
    return bn.g1_bytes(p).hex()


def _load_pp(bits):
    pp = ppm.load_pp(open(os.path.join(HERE, "zkatdlog_pp.json"), "rb").read())
    return pp if bits == 64 else pp.with_bit_length(bits)


def _retamper_rc(raw, j, fn):
    """apply fn to range proof j of a transfer/issue proof (DER round trip)"""
    sig, rc = der.unmarshal_values(raw)
    proofs = zkat.rc_deserialize(rc)
    fn(proofs[j])
    return der.values([sig, zkat.rc_serialize(proofs)])


def transfer_case(args):
    name, seed = args
    pp = _load_pp(64)
    rng = zkat.make_rng(seed)
    a, b = rng.getrandbits(62), rng.getrandbits(62)
    c = rng.randrange(a + b + 1)
    ins, outs = [a, b], [c, a + b - c]
    if name == "wrong_sum":                      # transfer_test.go:158-184 (90+60 != 110+45)
        ins, outs = [a, b], [c, a + b - c + 5]
    elif name == "out_of_range_index1":          # output 1 >= 2^64: its range proof fails
        ins = [(1 << 63) + 7, (1 << 63) + 9]
        outs = [10, (1 << 64) + 6]
    inbf = [rng.randrange(bn.R) for _ in ins]
    outbf = [rng.randrange(bn.R) for _ in outs]
    incom = [zkat.token_commit(pp.ped, T, v, x) for v, x in zip(ins, inbf)]
    outcom = [zkat.token_commit(pp.ped, T, v, x) for v, x in zip(outs, outbf)]
    prover_in = list(incom)
    verifier_in = list(incom)
    if name == "tas_wrong_type":                 # typeandsum_test.go:87-99: prover.Inputs[0] of type XYZ
        prover_in[0] = zkat.token_commit(pp.ped, b"XYZ", ins[0], inbf[0])
    elif name == "tas_wrong_values":             # :100-112: prover.Inputs[0] commits to another value
        prover_in[0] = zkat.token_commit(pp.ped, T, (ins[0] + 20) % (1 << 64), inbf[0])
    elif name == "tas_wrong_bf":                 # :127-141: verifier.Inputs[0] with another blinding factor
        verifier_in[0] = zkat.token_commit(pp.ped, T, ins[0], rng.randrange(bn.R))
    raw = zkat.transfer_prove(pp, [(v, x, T) for v, x in zip(ins, inbf)], [(v, x, T) for v, x in zip(outs, outbf)],
                              prover_in, outcom, rng)
    if name == "tampered_T1_index0":
        raw = _retamper_rc(raw, 0, lambda p: setattr(p.data, "T1", bn.g1_add(p.data.T1, pp.ped[1])))
    elif name == "tampered_L3_index1":
        raw = _retamper_rc(raw, 1, lambda p: p.ipa.L.__setitem__(3, bn.g1_add(p.ipa.L[3], pp.ped[1])))
    elif name == "tampered_delta_index1":
        raw = _retamper_rc(raw, 1, lambda p: setattr(p.data, "Delta", (p.data.Delta + 1) % bn.R))
    elif name == "tampered_right_index0":
        raw = _retamper_rc(raw, 0, lambda p: setattr(p.ipa, "Right", (p.ipa.Right + 3) % bn.R))
    err, idx = zkat.transfer_verify(pp, verifier_in, outcom, raw)
    return {"name": name, "bits": 64, "inputs": [pt(p) for p in verifier_in], "outputs": [pt(p) for p in outcom],
            "proof": raw.hex(), "expect": err, "index": idx}


def issue_case(args):
    name, seed = args
    pp = _load_pp(32)
    rng = zkat.make_rng(seed)
    vals = [rng.getrandbits(32) for _ in range(16)]
    bfs = [rng.randrange(bn.R) for _ in vals]
    toks = [zkat.token_commit(pp.ped, T, v, x) for v, x in zip(vals, bfs)]
    raw = zkat.issue_prove(pp, [(v, x, T) for v, x in zip(vals, bfs)], toks, rng)
    if name == "token5_other_value":
        toks[5] = zkat.token_commit(pp.ped, T, (vals[5] + 1) % (1 << 32), bfs[5])
    elif name == "tampered_challenge":
        st_raw, rc_raw = der.unmarshal_values(raw)
        st = zkat.SameType.deserialize(st_raw)
        st.Chal = (st.Chal + 1) % bn.R
        raw = der.values([st.serialize(), rc_raw])
    elif name == "tampered_L2_index11":
        raw = _retamper_rc(raw, 11, lambda p: p.ipa.L.__setitem__(2, bn.g1_add(p.ipa.L[2], pp.ped[2])))
    err, idx = zkat.issue_verify(pp, toks, raw)
    return {"name": name, "bits": 32, "tokens": [pt(p) for p in toks], "proof": raw.hex(), "expect": err,
            "index": idx}


TRANSFERS = [("honest", 0xF7A50001), ("honest_b", 0xF7A50011), ("wrong_sum", 0xF7A50002),
             ("out_of_range_index1", 0xF7A50003), ("tampered_T1_index0", 0xF7A50004),
             ("tampered_L3_index1", 0xF7A50005), ("tampered_delta_index1", 0xF7A50006),
             ("tampered_right_index0", 0xF7A50007), ("tas_wrong_type", 0xF7A50008),
             ("tas_wrong_values", 0xF7A50009), ("tas_wrong_bf", 0xF7A5000A)]
ISSUES = [("honest", 0xF7A50021), ("token5_other_value", 0xF7A50022), ("tampered_challenge", 0xF7A50023),
          ("tampered_L2_index11", 0xF7A50024)]


def main():
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        tr = pool.map_async(transfer_case, TRANSFERS)
        iss = pool.map_async(issue_case, ISSUES)
        out = {"transfers": tr.get(), "issues": iss.get()}
    with open(os.path.join(HERE, "headline_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    for c in out["transfers"] + out["issues"]:
        print(c["bits"], c["name"], c["expect"], c["index"])


if __name__ == "__main__":
    main()
