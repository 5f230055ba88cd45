"""Reference-order restatement of the zkatdlog (nogh v1) proof system
(oracle; test infrastructure only).

Every function cites the reference file:line it follows (paths relative to
token/core/zkatdlog/nogh/v1/crypto/ unless stated).  Verifiers run in the
reference's exact operation order and return the reference's error string
(``None`` on success); ``trace`` dicts record every exact intermediate
(challenges, H'_i, com, per-round C) so the GPU path can be checked
intermediate-by-intermediate, not only by verdict.
"""
import random

from . import bn254 as bn
from . import der

R = bn.R
SEP = b"||"  # common/array.go:19


class Malformed(Exception):
    """Input on which the reference returns a deserialization error or
    panics (nil dereference / index out of range).  The product maps both to
    FTS_E_MALFORMED (documented divergence for the panic cases)."""


# ---------------------------------------------------------------- transcript
def g1_array_bytes(points):
    """(*G1Array).Bytes, common/array.go:25-36: lowercase hex of each 64-byte
    point joined with "||"."""
    for p in points:
        if p is False:
            raise Malformed("failed to marshal array of G1")
    return SEP.join(bn.g1_bytes(p).hex().encode() for p in points)


# ------------------------------------------------------------ element codec
class _El:
    """a serialised mathlib element: G1 or Zr"""


def _g1_el(p):
    return der.element(1, bn.g1_bytes(p))


def _zr_el(z):
    return der.element(1, bn.zr_bytes(z))


def _g1_arr_el(ps):
    return der.element(1, der.values([bn.g1_bytes(p) for p in ps]))


def _zr_arr_el(zs):
    return der.element(1, der.values([bn.zr_bytes(z) for z in zs]))


def marshal_math(*elements):
    """asn1.MarshalMath, core/common/encoding/asn1/asn1.go:95-112"""
    return der.values(list(elements))


class Unmarshaller:
    """asn1.go:114-230.  NextX returns None once the values are exhausted."""

    def __init__(self, raw):
        try:
            self.v = der.unmarshal_values(raw)
        except der.DerError as e:
            raise Malformed("failed to unmarshal values: %s" % e)
        self.i = 0

    def _next(self):
        if self.i >= len(self.v):
            return None
        try:
            cid, raw = der.unmarshal_element(self.v[self.i])
        except der.DerError as e:
            raise Malformed("failed to unmarshal element: %s" % e)
        if cid != 1:
            # mathlib.Curves[cid]: another curve or an index panic
            raise Malformed("unsupported curve id %d" % cid)
        self.i += 1
        return raw

    def g1(self):
        raw = self._next()
        if raw is None:
            return False  # Go nil
        try:
            return bn.g1_from_bytes(raw)
        except bn.PointError as e:
            raise Malformed(str(e))

    def zr(self):
        raw = self._next()
        if raw is None:
            return None
        return bn.zr_from_bytes(raw)

    def _arr(self):
        raw = self._next()
        if raw is None:
            return None
        try:
            return der.unmarshal_values_strict(raw)
        except der.DerError as e:
            raise Malformed(str(e))

    def zr_array(self):
        vals = self._arr()
        return None if vals is None else [bn.zr_from_bytes(x) for x in vals]

    def g1_array(self):
        vals = self._arr()
        if vals is None:
            return None
        try:
            return [bn.g1_from_bytes(x) for x in vals]
        except bn.PointError as e:
            raise Malformed(str(e))


def _unmarshal_pair(raw):
    """asn1.Unmarshal[S](raw, a, b) (asn1.go:57-76): exactly 2 values; empty
    values are skipped (left as freshly allocated objects)."""
    try:
        vals = der.unmarshal_values(raw)
    except der.DerError as e:
        raise Malformed("failed to unmarshal values: %s" % e)
    if len(vals) != 2:
        raise Malformed("number of values does not match number of values")
    return vals


# ------------------------------------------------------------ proof objects
class RangeProofData:
    """rp/bulletproof.go:16-83"""
    __slots__ = ("T1", "T2", "Tau", "C", "D", "Delta", "InnerProduct")

    def __init__(self, **kw):
        for s in self.__slots__:
            setattr(self, s, kw.get(s, False if s in ("T1", "T2", "C", "D") else None))

    def serialize(self):
        return marshal_math(_g1_el(self.T1), _g1_el(self.T2), _zr_el(self.Tau), _g1_el(self.C),
                            _g1_el(self.D), _zr_el(self.Delta), _zr_el(self.InnerProduct))

    @classmethod
    def deserialize(cls, raw):
        u = Unmarshaller(raw)
        d = cls()
        d.T1 = u.g1(); d.T2 = u.g1(); d.Tau = u.zr(); d.C = u.g1(); d.D = u.g1()
        d.Delta = u.zr(); d.InnerProduct = u.zr()
        return d


class IPA:
    """rp/ipa.go:18-67"""

    def __init__(self, Left=None, Right=None, L=None, R=None):
        self.Left, self.Right, self.L, self.R = Left, Right, L, R

    def serialize(self):
        return marshal_math(_zr_el(self.Left), _zr_el(self.Right), _g1_arr_el(self.L), _g1_arr_el(self.R))

    @classmethod
    def deserialize(cls, raw):
        u = Unmarshaller(raw)
        return cls(u.zr(), u.zr(), u.g1_array(), u.g1_array())


class RangeProof:
    """rp/bulletproof.go:86-101"""

    def __init__(self, data=None, ipa=None):
        self.data, self.ipa = data, ipa

    def serialize(self):
        return der.values([self.data.serialize(), self.ipa.serialize()])

    @classmethod
    def deserialize(cls, raw):
        vals = _unmarshal_pair(raw)
        rp = cls(RangeProofData(), IPA())
        if vals[0]:
            rp.data = RangeProofData.deserialize(vals[0])
        if vals[1]:
            rp.ipa = IPA.deserialize(vals[1])
        return rp


def rc_serialize(proofs):
    """RangeCorrectness.Serialize, rp/rangecorrectness.go:19-25 (double Values wrap)"""
    return der.values([der.values([p.serialize() for p in proofs])])


def rc_deserialize(raw):
    """rp/rangecorrectness.go:27-40 via asn1 array/UnmarshalTo (asn1.go:78-93,269-290)"""
    try:
        outer = der.unmarshal_values(raw)
    except der.DerError as e:
        raise Malformed("failed to unmarshal proofs: %s" % e)
    if len(outer) != 1:
        raise Malformed("failed to unmarshal proofs: number of values does not match")
    if not outer[0]:
        return []
    try:
        inner = der.unmarshal_values(outer[0])
    except der.DerError as e:
        raise Malformed("failed to unmarshal proofs: %s" % e)
    return [RangeProof.deserialize(x) for x in inner]


# ------------------------------------------------------------------- prover
def _commit_vector(left, right, lg, rg):
    """rp/ipa.go:366-373"""
    com = None
    for i in range(len(left)):
        com = bn.g1_add(com, bn.g1_mul(lg[i], left[i]))
        com = bn.g1_add(com, bn.g1_mul(rg[i], right[i]))
    return com


def _ip(a, b):
    return sum(x * y for x, y in zip(a, b)) % R


def _reduce_generators(lg, rg, x, xinv):
    """rp/ipa.go:343-356"""
    m = len(lg) // 2
    nl = [bn.g1_add(bn.g1_mul(lg[i], xinv), bn.g1_mul(lg[i + m], x)) for i in range(m)]
    nr = [bn.g1_add(bn.g1_mul(rg[i], x), bn.g1_mul(rg[i + m], xinv)) for i in range(m)]
    return nl, nr


def ipa_prove(ip, left, right, Q, lg, rg, com, rounds):
    """rp/ipa.go:158-186 + reduce :267-322"""
    arr = g1_array_bytes(rg + lg + [Q, com])
    x = bn.hash_to_zr(der.marshal_std_bytes_list([arr, SEP, bn.zr_bytes(ip)]))
    C = bn.g1_add(bn.g1_mul(Q, x * ip % R), com)
    X = bn.g1_mul(Q, x)
    Ls, Rs = [], []
    for _ in range(rounds):
        n = len(lg) // 2
        lip = _ip(left[:n], right[n:])
        rip = _ip(left[n:], right[:n])
        Lj = bn.g1_add(_commit_vector(left[:n], right[n:], lg[n:], rg[:n]), bn.g1_mul(X, lip))
        Rj = bn.g1_add(_commit_vector(left[n:], right[:n], lg[:n], rg[n:]), bn.g1_mul(X, rip))
        Ls.append(Lj)
        Rs.append(Rj)
        xj = bn.hash_to_zr(g1_array_bytes([Lj, Rj]))
        xinv = pow(xj, R - 2, R)
        lg, rg = _reduce_generators(lg, rg, xj, xinv)
        left = [(left[i] * xj + left[i + n] * xinv) % R for i in range(n)]
        right = [(right[i] * xinv + right[i + n] * xj) % R for i in range(n)]
    return IPA(left[0], right[0], Ls, Rs)


def rp_prove(com, value, commit_gens, bf, lg, rg, P, Q, rounds, n, rng):
    """rangeProver.Prove + preprocess, rp/bulletproof.go:209-249,336-466"""
    G, H = commit_gens
    rnd = lambda: rng.randrange(R)
    left = [(value >> i) & 1 for i in range(n)]
    right = [(b - 1) % R for b in left]
    rho, eta = rnd(), rnd()
    randL, randR = [], []
    for i in range(n):
        randL.append(rnd())
        randR.append(rnd())
    C = bn.g1_add(_commit_vector(left, right, lg, rg), bn.g1_mul(P, rho))
    D = bn.g1_add(_commit_vector(randL, randR, lg, rg), bn.g1_mul(P, eta))
    y = bn.hash_to_zr(g1_array_bytes([C, D, com]))
    z = bn.hash_to_zr(bn.zr_bytes(y))
    z2 = z * z % R
    lp, rpv, rrp, zp = [], [], [], []
    yi = 1
    for i in range(n):
        if i:
            yi = yi * y % R
        lp.append((left[i] - z) % R)
        rpv.append((right[i] + z) * yi % R)
        rrp.append(randR[i] * yi % R)
        zp.append(z2 * pow(2, i, R) % R)
    t1 = (_ip(lp, rrp) + _ip(rpv, randL) + _ip(zp, randL)) % R
    tau1 = rnd()
    T1 = bn.g1_add(bn.g1_mul(G, t1), bn.g1_mul(H, tau1))
    t2 = _ip(randL, rrp)
    tau2 = rnd()
    T2 = bn.g1_add(bn.g1_mul(G, t2), bn.g1_mul(H, tau2))
    x = bn.hash_to_zr(g1_array_bytes([T1, T2]))
    L = [(lp[i] + x * randL[i]) % R for i in range(n)]
    Rv = [(rpv[i] + x * rrp[i] + zp[i]) % R for i in range(n)]
    tau = (x * tau1 + tau2 * x * x + z2 * bf) % R
    delta = (rho + eta * x) % R
    data = RangeProofData(T1=T1, T2=T2, C=C, D=D, Tau=tau, Delta=delta)
    yinv = pow(y, R - 2, R)
    rgp = [bn.g1_mul(rg[i], pow(yinv, i, R)) for i in range(n)]
    comv = _commit_vector(L, Rv, lg, rgp)
    data.InnerProduct = _ip(L, Rv)
    ipa = ipa_prove(data.InnerProduct, L, Rv, Q, lg, rgp, comv, rounds)
    return RangeProof(data, ipa)


# ----------------------------------------------------------------- verifier
def ipa_verify(ip, Q, lg, rg, com, rounds, proof, trace=None):
    """(*ipaVerifier).Verify, rp/ipa.go:190-262"""
    if proof.Left is None or proof.Right is None:
        return "invalid IPA proof: nil elements"
    if proof.L is None or proof.R is None:
        Ln = 0 if proof.L is None else len(proof.L)
        Rn = 0 if proof.R is None else len(proof.R)
    else:
        Ln, Rn = len(proof.L), len(proof.R)
    if Ln != Rn or Ln != rounds:
        return "invalid IPA proof"
    arr = g1_array_bytes(rg + lg + [Q, com])
    raw = der.marshal_std_bytes_list([arr, SEP, bn.zr_bytes(ip)])
    x = bn.hash_to_zr(raw)
    C = bn.g1_add(bn.g1_mul(Q, x * ip % R), com)
    X = bn.g1_mul(Q, x)
    if trace is not None:
        trace["x0"] = x
        trace["x0_transcript_len"] = len(raw)
        trace["C0"] = C
        trace["xj"] = []
        trace["Cj"] = []
    for i in range(rounds):
        if proof.L[i] is False or proof.R[i] is False:
            return "invalid IPA proof: nil elements"
        xj = bn.hash_to_zr(g1_array_bytes([proof.L[i], proof.R[i]]))
        xinv = pow(xj, R - 2, R)
        xsq = xj * xj % R
        xsqinv = pow(xsq, R - 2, R)
        Cp = bn.g1_add(bn.g1_add(bn.g1_mul(proof.L[i], xsq), C), bn.g1_mul(proof.R[i], xsqinv))
        C = Cp
        lg, rg = _reduce_generators(lg, rg, xj, xinv)
        if trace is not None:
            trace["xj"].append(xj)
            trace["Cj"].append(C)
    Cp = bn.g1_mul(lg[0], proof.Left)
    Cp = bn.g1_add(Cp, bn.g1_mul(rg[0], proof.Right))
    Cp = bn.g1_add(Cp, bn.g1_mul(X, proof.Left * proof.Right % R))
    if trace is not None:
        trace["G_fin"] = lg[0]
        trace["H_fin"] = rg[0]
        trace["final_lhs"] = Cp
    if Cp != C:
        return "invalid IPA"
    return None


def rp_verify(V, commit_gens, lg, rg, P, Q, rounds, n, rp, trace=None):
    """(*rangeVerifier).Verify + verifyIPA, rp/bulletproof.go:252-333,469-509"""
    d = rp.data
    if d.InnerProduct is None or d.C is False or d.D is False:
        return "invalid range proof: nil elements"
    if d.T1 is False or d.T2 is False:
        return "invalid range proof: nil elements"
    if d.Tau is None or d.Delta is None:
        return "invalid range proof: nil elements"
    if rp.ipa is None:
        return "invalid range proof: nil elements"
    G, H = commit_gens
    x = bn.hash_to_zr(g1_array_bytes([d.T1, d.T2]))
    x2 = x * x % R
    y = bn.hash_to_zr(g1_array_bytes([d.C, d.D, V]))
    z = bn.hash_to_zr(bn.zr_bytes(y))
    z2 = z * z % R
    z3 = z2 * z % R
    ypow = []
    ipy = ip2 = 0
    p2 = 1
    for i in range(len(rg)):
        if i == 0:
            ypow.append(1)
            p2 = 1
        else:
            ypow.append(y * ypow[-1] % R)
            p2 = 2 * p2 % R
        ipy = (ipy + ypow[i]) % R
        ip2 = (ip2 + p2) % R
    pol = ((z - z2) * ipy - z3 * ip2) % R
    com = bn.g1_mul(G, d.InnerProduct)
    com = bn.g1_add(com, bn.g1_mul(H, d.Tau))
    com = bn.g1_sub(com, bn.g1_mul(d.T1, x))
    com = bn.g1_sub(com, bn.g1_mul(d.T2, x2))
    comp = bn.g1_mul(V, z2)
    comp = bn.g1_add(comp, bn.g1_mul(G, pol))
    if trace is not None:
        trace.update(x=x, y=y, z=z, polEval=pol, E1_lhs=com, E1_rhs=comp)
    if com != comp:
        return "invalid range proof"
    # verifyIPA (bulletproof.go:469-509)
    c = bn.g1_add(bn.g1_mul(d.D, x), d.C)
    rgp = []
    for i in range(len(lg)):
        c = bn.g1_sub(c, bn.g1_mul(lg[i], z))
        yinv = pow(ypow[i], R - 2, R)
        zi = (z * ypow[i] + z2 * pow(2, i, R)) % R
        rgp.append(bn.g1_mul(rg[i], yinv))
        c = bn.g1_add(c, bn.g1_mul(rgp[i], zi))
    c = bn.g1_sub(c, bn.g1_mul(P, d.Delta))
    if trace is not None:
        trace["Hprime"] = rgp
        trace["com"] = c
    return ipa_verify(d.InnerProduct, Q, lg, rgp, c, rounds, rp.ipa, trace)


def rc_verify(coms, ped_rp, lg, rg, P, Q, n, rounds, proofs, traces=None):
    """RangeCorrectnessVerifier.Verify, rp/rangecorrectness.go:137-162.
    -> (error string or None, failing index or -1)"""
    if len(proofs) != len(coms):
        return "invalid range proof", -1
    for i, p in enumerate(proofs):
        tr = {} if traces is not None else None
        err = rp_verify(coms[i], ped_rp, lg, rg, P, Q, rounds, n, p, tr)
        if traces is not None:
            traces.append(tr)
        if err:
            return "invalid range proof at index %d: %s" % (i, err), i
    return None, -1


# ---------------------------------------------------------- TypeAndSum (transfer)
class TypeAndSumProof:
    """transfer/typeandsum.go:19-93"""

    def __init__(self, CT=False, ibf=None, iv=None, Type=None, TBF=None, EqSum=None, Chal=None):
        self.CT, self.ibf, self.iv, self.Type, self.TBF, self.EqSum, self.Chal = CT, ibf, iv, Type, TBF, EqSum, Chal

    def serialize(self):
        return marshal_math(_g1_el(self.CT), _zr_arr_el(self.ibf), _zr_arr_el(self.iv), _zr_el(self.Type),
                            _zr_el(self.TBF), _zr_el(self.EqSum), _zr_el(self.Chal))

    @classmethod
    def deserialize(cls, raw):
        u = Unmarshaller(raw)
        return cls(u.g1(), u.zr_array(), u.zr_array(), u.zr(), u.zr(), u.zr(), u.zr())


def tas_prove(ped, inputs, outputs, ct, in_vals, in_bfs, out_bfs, type_zr, type_bf, rng):
    """TypeAndSumProver.Prove, transfer/typeandsum.go:189-356"""
    rnd = lambda: rng.randrange(R)
    r_ttype, r_tbf = rnd(), rnd()
    com_ct = bn.g1_add(bn.g1_mul(ped[0], r_ttype), bn.g1_mul(ped[2], r_tbf))
    r_iv, r_ibf, com_in = [], [], []
    for i in range(len(inputs)):
        r_iv.append(rnd())
        r_ibf.append(rnd())
        com_in.append(bn.g1_add(bn.g1_mul(ped[1], r_iv[i]), bn.g1_mul(ped[2], r_ibf[i])))
    r_sum = rnd()
    com_sum = bn.g1_mul(ped[2], r_sum)
    ins, outs = [], []
    s = None
    for i in inputs:
        ins.append(bn.g1_sub(i, ct))
        s = bn.g1_add(s, ins[-1])
    for o in outputs:
        outs.append(bn.g1_sub(o, ct))
        s = bn.g1_sub(s, outs[-1])
    raw = g1_array_bytes(com_in + [com_ct, com_sum] + ins + outs + [ct, s])
    chal = bn.hash_to_zr(raw)
    p = TypeAndSumProof(CT=ct, Chal=chal)
    p.Type = (chal * type_zr + r_ttype) % R
    p.TBF = (chal * type_bf + r_tbf) % R
    p.iv, p.ibf = [], []
    sum_bf = 0
    for i in range(len(inputs)):
        p.iv.append((chal * in_vals[i] + r_iv[i]) % R)
        t = (in_bfs[i] - type_bf) % R
        p.ibf.append((chal * t + r_ibf[i]) % R)
        sum_bf = (sum_bf + t) % R
    for i in range(len(outputs)):
        sum_bf = (sum_bf - (out_bfs[i] - type_bf)) % R
    p.EqSum = (chal * sum_bf + r_sum) % R
    return p


def tas_verify(ped, inputs, outputs, stp, trace=None):
    """(*TypeAndSumVerifier).Verify, transfer/typeandsum.go:230-277"""
    if stp.TBF is None or stp.Type is None or stp.CT is False or stp.EqSum is None:
        return "invalid sum and type proof"
    if stp.Chal is None or stp.iv is None or stp.ibf is None \
            or len(stp.iv) < len(inputs) or len(stp.ibf) < len(inputs):
        raise Malformed("reference panics: nil/short TypeAndSum fields")
    ins, outs, incoms = [], [], []
    s = None
    for i in range(len(inputs)):
        ins.append(bn.g1_sub(inputs[i], stp.CT))
        s = bn.g1_add(s, ins[i])
        c = bn.g1_mul(ped[1], stp.iv[i])
        c = bn.g1_add(c, bn.g1_mul(ped[2], stp.ibf[i]))
        c = bn.g1_sub(c, bn.g1_mul(ins[i], stp.Chal))
        incoms.append(c)
    for o in outputs:
        outs.append(bn.g1_sub(o, stp.CT))
        s = bn.g1_sub(s, outs[-1])
    sumcom = bn.g1_sub(bn.g1_mul(ped[2], stp.EqSum), bn.g1_mul(s, stp.Chal))
    typecom = bn.g1_add(bn.g1_mul(ped[0], stp.Type), bn.g1_mul(ped[2], stp.TBF))
    typecom = bn.g1_sub(typecom, bn.g1_mul(stp.CT, stp.Chal))
    raw = g1_array_bytes(incoms + [typecom, sumcom] + ins + outs + [stp.CT, s])
    chal = bn.hash_to_zr(raw)
    if trace is not None:
        trace.update(inComs=incoms, typeCom=typecom, sumCom=sumcom, sum=s, chal=chal, transcript_len=len(raw))
    if chal != stp.Chal:  # Zr.Equals: raw integer compare
        return "invalid sum and type proof"
    return None


# ------------------------------------------------------------ transfer proof
def transfer_serialize(tas, proofs):
    """transfer.Proof.Serialize, transfer/transfer.go:29-34 (nil RC -> empty)"""
    return der.values([tas.serialize(), rc_serialize(proofs) if proofs is not None else b""])


def transfer_verify(pp, inputs, outputs, raw, traces=None):
    """transfer.NewVerifier + (*Verifier).Verify, transfer/transfer.go:49-60,153-197.
    -> (error string or None, failing range index or -1)"""
    try:
        vals = _unmarshal_pair(raw)
        tas = TypeAndSumProof()
        proofs = []
        if vals[0]:
            tas = TypeAndSumProof.deserialize(vals[0])
        if vals[1]:
            proofs = rc_deserialize(vals[1])
    except Malformed as e:
        return "invalid transfer proof: %s" % e, -1
    tsp_err = tas_verify(pp.ped, inputs, outputs, tas)
    range_err, idx = None, -1
    if len(inputs) != 1 or len(outputs) != 1:
        if tas.CT is False:
            raise Malformed("reference panics: nil CommitmentToType")
        coms = [bn.g1_sub(o, tas.CT) for o in outputs]
        range_err, idx = rc_verify(coms, pp.ped[1:], pp.left, pp.right, pp.P, pp.Q, pp.bit_length,
                                   pp.rounds, proofs, traces)
    if tsp_err:
        return "invalid transfer proof: %s" % tsp_err, -1
    return range_err, idx


def transfer_prove(pp, in_tw, out_tw, inputs, outputs, rng):
    """transfer.NewProver + Prove, transfer/transfer.go:69-150.
    tw = (value, blinding factor, type bytes)"""
    type_zr = bn.hash_to_zr(in_tw[0][2])
    ct = bn.g1_mul(pp.ped[0], type_zr)
    type_bf = rng.randrange(R)
    ct = bn.g1_add(ct, bn.g1_mul(pp.ped[2], type_bf))
    proofs = None
    if len(in_tw) != 1 or len(out_tw) != 1:
        coms = [bn.g1_sub(o, ct) for o in outputs]
        proofs = [rp_prove(coms[i], out_tw[i][0], pp.ped[1:], (out_tw[i][1] - type_bf) % R, pp.left,
                           pp.right, pp.P, pp.Q, pp.rounds, pp.bit_length, rng) for i in range(len(outputs))]
    tas = tas_prove(pp.ped, inputs, outputs, ct, [t[0] for t in in_tw], [t[1] for t in in_tw],
                    [t[1] for t in out_tw], type_zr, type_bf, rng)
    return transfer_serialize(tas, proofs)


# ------------------------------------------------------------ SameType (issue)
class SameType:
    """issue/sametype.go:19-64"""

    def __init__(self, Type=None, BF=None, Chal=None, CT=False):
        self.Type, self.BF, self.Chal, self.CT = Type, BF, Chal, CT

    def serialize(self):
        return marshal_math(_zr_el(self.Type), _zr_el(self.BF), _zr_el(self.Chal), _g1_el(self.CT))

    @classmethod
    def deserialize(cls, raw):
        u = Unmarshaller(raw)
        return cls(u.zr(), u.zr(), u.zr(), u.g1())


def st_prove(ped, type_bytes, bf, ct, rng):
    """SameTypeProver.Prove, issue/sametype.go:103-148"""
    t = bn.hash_to_zr(type_bytes)
    r_t, r_bf = rng.randrange(R), rng.randrange(R)
    com = bn.g1_add(bn.g1_mul(ped[0], r_t), bn.g1_mul(ped[2], r_bf))
    chal = bn.hash_to_zr(g1_array_bytes([ct, com]))
    return SameType((chal * t + r_t) % R, (chal * bf + r_bf) % R, chal, ct)


def st_verify(ped, proof, trace=None):
    """(*SameTypeVerifier).Verify, issue/sametype.go:167-183"""
    if proof.Type is None or proof.BF is None or proof.Chal is None or proof.CT is False:
        raise Malformed("reference panics: nil SameType fields")
    com = bn.g1_add(bn.g1_mul(ped[0], proof.Type), bn.g1_mul(ped[2], proof.BF))
    com = bn.g1_sub(com, bn.g1_mul(proof.CT, proof.Chal))
    chal = bn.hash_to_zr(g1_array_bytes([proof.CT, com]))
    if trace is not None:
        trace.update(com=com, chal=chal)
    if chal != proof.Chal:
        return "invalid same type proof"
    return None


def issue_prove(pp, tw, tokens, rng):
    """issue.NewProver + Prove, issue/prover.go:46-112"""
    t = bn.hash_to_zr(tw[0][2])
    ct = bn.g1_mul(pp.ped[0], t)
    bf = rng.randrange(R)
    ct = bn.g1_add(ct, bn.g1_mul(pp.ped[2], bf))
    st = st_prove(pp.ped, tw[0][2], bf, ct, rng)
    coms = [bn.g1_sub(tok, ct) for tok in tokens]
    proofs = [rp_prove(coms[i], tw[i][0], pp.ped[1:], (tw[i][1] - bf) % R, pp.left, pp.right, pp.P,
                       pp.Q, pp.rounds, pp.bit_length, rng) for i in range(len(tokens))]
    return der.values([st.serialize(), rc_serialize(proofs)])


def issue_verify(pp, tokens, raw, traces=None):
    """issue.NewVerifier + (*Verifier).Verify, issue/verifier.go:24-57"""
    try:
        vals = _unmarshal_pair(raw)
        st = SameType()
        proofs = []
        if vals[0]:
            st = SameType.deserialize(vals[0])
        if vals[1]:
            proofs = rc_deserialize(vals[1])
    except Malformed as e:
        return str(e), -1
    err = st_verify(pp.ped, st)
    if err:
        return "invalid issue proof: %s" % err, -1
    coms = [bn.g1_sub(tok, st.CT) for tok in tokens]
    err, idx = rc_verify(coms, pp.ped[1:], pp.left, pp.right, pp.P, pp.Q, pp.bit_length, pp.rounds,
                         proofs, traces)
    if err:
        return "invalid issue proof: %s" % err, idx
    return None, -1


# ------------------------------------------------------------------- tokens
def token_commit(ped, type_bytes, value, bf):
    """token.commit / computeTokens, crypto/token/token.go:109-130,208-217"""
    c = bn.g1_mul(ped[0], bn.hash_to_zr(type_bytes))
    c = bn.g1_add(c, bn.g1_mul(ped[1], value))
    return bn.g1_add(c, bn.g1_mul(ped[2], bf))


def make_rng(seed):
    return random.Random(seed)


# ------------------------------------------------------------------ auditor
def inspect_output(ped, com_bytes, type_bytes, value_bytes, bf_bytes, index=0):
    """Auditor.InspectOutput's opening check, crypto/audit/auditor.go:226-238
    (commit() :412-418): tokenComm = HashToZr(type) ped0 + value ped1 + bf ped2,
    compared with token.Data.  Returns the reference error string or None.
    ``com_bytes`` goes through NewG1FromBytes (PointError -> "malformed");
    value/bf through NewZrFromBytes (unreduced; G1.Mul uses them mod r).
    A None field is the nil case the library reports as FTS_E_MALFORMED."""
    if com_bytes is None or value_bytes is None or bf_bytes is None:
        return "malformed"
    try:
        com = bn.g1_from_bytes(com_bytes)
    except bn.PointError:
        return "malformed"
    c = token_commit(ped, type_bytes, bn.zr_from_bytes(value_bytes) % R, bn.zr_from_bytes(bf_bytes) % R)
    if c != com:
        return "output at index [%d] does not match the provided opening" % index
    return None
