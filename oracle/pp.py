"""Public-parameter loader (oracle; test infrastructure only).

Restates ``PublicParams.Deserialize`` (token/core/zkatdlog/nogh/v1/crypto/
setup.go:319-372): a JSON container ``{"identifier", "raw"}``
(core/common/encoding/pp/pp.go:16-30) whose ``raw`` is the protobuf
``nogh.PublicParameters`` (nogh/protos/noghpp.proto:25-44); every G1 is a
``nogh.G1{raw}`` holding mathlib's JSON ``{"curve":1,"element":b64}``
(nogh/protos-go/utils/proto.go:22-50).
"""
import base64
import json
from dataclasses import dataclass, field

from . import bn254


def _varint(b, i):
    shift = 0
    v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return v, i


def pb_fields(b):
    """Decode one protobuf message into [(field_no, wire_type, value)]."""
    out = []
    i = 0
    while i < len(b):
        key, i = _varint(b, i)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 2:
            ln, i = _varint(b, i)
            v = bytes(b[i:i + ln])
            i += ln
        elif wt == 1:
            v = bytes(b[i:i + 8])
            i += 8
        elif wt == 5:
            v = bytes(b[i:i + 4])
            i += 4
        else:
            raise ValueError("unsupported wire type %d" % wt)
        out.append((fno, wt, v))
    return out


def _g1_from_proto(raw):
    f = pb_fields(raw)
    js = [v for (n, w, v) in f if n == 1]
    if not js:
        return None
    obj = json.loads(js[0])
    if obj.get("curve") != 1:
        raise ValueError("unsupported curve %r" % obj.get("curve"))
    return bn254.g1_from_bytes(base64.b64decode(obj["element"]))


@dataclass
class PublicParams:
    label: str = ""
    version: str = ""
    curve: int = 1
    ped: list = field(default_factory=list)          # PedersenGenerators (3)
    left: list = field(default_factory=list)         # RangeProofParams.LeftGenerators
    right: list = field(default_factory=list)        # RangeProofParams.RightGenerators
    P: tuple = None
    Q: tuple = None
    bit_length: int = 0
    rounds: int = 0
    max_token: int = 0
    precision: int = 0

    def with_bit_length(self, n):
        """Same generators truncated to n (labels do not depend on n:
        setup.go:392-402), as Setup(n) would derive them."""
        k = n.bit_length() - 1
        assert 1 << k == n and n <= len(self.left)
        return PublicParams(self.label, self.version, self.curve, list(self.ped),
                            self.left[:n], self.right[:n], self.P, self.Q, n, k,
                            (1 << n) - 1, n)


def load_pp(container_bytes, label="zkatdlog"):
    c = json.loads(container_bytes)
    if c["identifier"] != label:
        raise ValueError("invalid identifier")
    raw = base64.b64decode(c["raw"])
    pp = PublicParams()
    for (n, w, v) in pb_fields(raw):
        if n == 1:
            pp.label = v.decode()
        elif n == 2:
            pp.version = v.decode()
        elif n == 3:
            cf = pb_fields(v)
            pp.curve = cf[0][2] if cf else 0
        elif n == 4:
            pp.ped.append(_g1_from_proto(v))
        elif n == 5:
            for (m, w2, u) in pb_fields(v):
                if m == 1:
                    pp.left.append(_g1_from_proto(u))
                elif m == 2:
                    pp.right.append(_g1_from_proto(u))
                elif m == 3:
                    pp.P = _g1_from_proto(u)
                elif m == 4:
                    pp.Q = _g1_from_proto(u)
                elif m == 5:
                    pp.bit_length = u
                elif m == 6:
                    pp.rounds = u
        elif n == 9:
            pp.max_token = v
        elif n == 10:
            pp.precision = v
    return pp
