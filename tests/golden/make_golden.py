"""Generate the golden fixtures of tests/golden/ with the CPU oracle.

The reference holds no golden proofs (every proof test in it is randomised,
SURVEY §4/§8c); its only known-answer fixture is zkatdlog_pp.json (copied here
unchanged).  These vectors are produced by the oracle's restatement of the
reference provers/verifiers (oracle/zkat.py), seeded, and record verdicts,
the reference error strings and exact intermediates.

    python tests/golden/make_golden.py        # rewrites *_golden.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bn254 as bn, pp as ppm, zkat  # noqa: E402


def hx(b):
    return b.hex()


def pt(p):
    return bn.g1_bytes(p).hex()


def rp_case(pp, n, value, seed, tamper=None):
    rng = zkat.make_rng(seed)
    bf = rng.randrange(bn.R)
    V = bn.g1_add(bn.g1_mul(pp.ped[1], value), bn.g1_mul(pp.ped[2], bf))
    proof = zkat.rp_prove(V, value, pp.ped[1:], bf, pp.left, pp.right, pp.P, pp.Q, pp.rounds, n, rng)
    if tamper == "T1":
        proof.data.T1 = bn.g1_add(proof.data.T1, pp.ped[1])
    elif tamper == "L0":
        proof.ipa.L[0] = bn.g1_add(proof.ipa.L[0], pp.ped[1])
    elif tamper == "Left":
        proof.ipa.Left = (proof.ipa.Left + 1) % bn.R
    elif tamper == "ip":
        proof.data.InnerProduct = (proof.data.InnerProduct + 1) % bn.R
    raw = proof.serialize()
    tr = {}
    err = zkat.rp_verify(V, pp.ped[1:], pp.left, pp.right, pp.P, pp.Q, pp.rounds, n,
                         zkat.RangeProof.deserialize(raw), tr)
    case = {"bits": n, "value": value, "tamper": tamper, "commitment": pt(V), "proof": hx(raw), "expect": err,
            "x": tr.get("x"), "y": tr.get("y"), "z": tr.get("z"), "polEval": tr.get("polEval")}
    if "com" in tr:
        case.update(com=pt(tr["com"]), hprime=[pt(h) for h in tr["Hprime"]], x0=tr.get("x0"),
                    xj=tr.get("xj"))
    return {k: (str(v) if isinstance(v, int) and k in ("x", "y", "z", "polEval", "x0") else v)
            for k, v in case.items()}


def transfer_case(pp, ins, outs, seed, name):
    rng = zkat.make_rng(seed)
    ttype = b"ABC"
    inbf = [rng.randrange(bn.R) for _ in ins]
    outbf = [rng.randrange(bn.R) for _ in outs]
    incom = [zkat.token_commit(pp.ped, ttype, v, b) for v, b in zip(ins, inbf)]
    outcom = [zkat.token_commit(pp.ped, ttype, v, b) for v, b in zip(outs, outbf)]
    raw = zkat.transfer_prove(pp, [(v, b, ttype) for v, b in zip(ins, inbf)],
                              [(v, b, ttype) for v, b in zip(outs, outbf)], incom, outcom, rng)
    err, idx = zkat.transfer_verify(pp, incom, outcom, raw)
    return {"name": name, "bits": pp.bit_length, "inputs": [pt(p) for p in incom], "outputs": [pt(p) for p in outcom],
            "proof": hx(raw), "expect": err, "index": idx}


def issue_case(pp, vals, seed, name, tamper=None):
    rng = zkat.make_rng(seed)
    ttype = b"ABC"
    bfs = [rng.randrange(bn.R) for _ in vals]
    toks = [zkat.token_commit(pp.ped, ttype, v, b) for v, b in zip(vals, bfs)]
    raw = zkat.issue_prove(pp, [(v, b, ttype) for v, b in zip(vals, bfs)], toks, rng)
    if tamper == "chal":
        from oracle import der
        st_raw, rc_raw = der.unmarshal_values(raw)
        st = zkat.SameType.deserialize(st_raw)
        st.Chal = (st.Chal + 1) % bn.R
        raw = der.values([st.serialize(), rc_raw])
    err, idx = zkat.issue_verify(pp, toks, raw)
    return {"name": name, "bits": pp.bit_length, "tokens": [pt(p) for p in toks], "proof": hx(raw), "expect": err,
            "index": idx}


def main():
    pp64 = ppm.load_pp(open(os.path.join(HERE, "zkatdlog_pp.json"), "rb").read())
    rp = []
    pp8 = pp64.with_bit_length(8)
    rp.append(rp_case(pp8, 8, 115, 1))                     # bulletproof_test.go:18-53 (value 115)
    rp.append(rp_case(pp8, 8, 0, 2))
    rp.append(rp_case(pp8, 8, 255, 3))
    rp.append(rp_case(pp8, 8, 260, 4))                     # out of range -> "invalid range proof"
    rp.append(rp_case(pp8, 8, 77, 5, "T1"))
    rp.append(rp_case(pp8, 8, 77, 6, "L0"))
    rp.append(rp_case(pp8, 8, 77, 7, "Left"))
    rp.append(rp_case(pp8, 8, 77, 8, "ip"))
    pp16 = pp64.with_bit_length(16)
    rp.append(rp_case(pp16, 16, 40000, 9))
    pp32 = pp64.with_bit_length(32)
    rp.append(rp_case(pp32, 32, 3000000000, 10))
    rp.append(rp_case(pp64, 64, (1 << 64) - 1, 11))
    rp.append(rp_case(pp64, 64, 0xF7A50002, 12))
    rp.append(rp_case(pp64, 64, 12345, 13, "L0"))
    with open(os.path.join(HERE, "rp_golden.json"), "w") as f:
        json.dump(rp, f, indent=1)
    tr = [
        transfer_case(pp16, [220, 60], [260, 20], 21, "honest_2in_2out"),          # transfer_test.go:130-156
        transfer_case(pp16, [90, 60], [110, 45], 22, "wrong_sum"),                # :158-184
        transfer_case(pp8, [220, 60], [260, 20], 23, "out_of_range_8bit"),        # :109-118
        transfer_case(pp16, [500], [500], 24, "ownership_1in_1out"),              # transfer.go:55 (no RC)
        transfer_case(pp16, [100, 200, 300], [600], 25, "honest_3in_1out"),
    ]
    with open(os.path.join(HERE, "transfer_golden.json"), "w") as f:
        json.dump(tr, f, indent=1)
    iss = [
        issue_case(pp16, [10, 20], 31, "honest_2"),                               # issue_test.go:15-22
        issue_case(pp16, [7], 32, "tampered_challenge", tamper="chal"),
        issue_case(pp8, [300, 1], 33, "out_of_range_8bit"),
    ]
    with open(os.path.join(HERE, "issue_golden.json"), "w") as f:
        json.dump(iss, f, indent=1)
    print("rp", [c["expect"] for c in rp])
    print("transfer", [(c["name"], c["expect"]) for c in tr])
    print("issue", [(c["name"], c["expect"]) for c in iss])


if __name__ == "__main__":
    main()
