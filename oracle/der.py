"""DER codec restating the subset of Go encoding/asn1 used by
token/core/common/encoding/asn1/asn1.go (oracle; test infrastructure only).

Shapes (asn1.go:27-34):
  Values  = SEQUENCE { SEQUENCE OF OCTET STRING }
  Element = SEQUENCE { INTEGER curveID, OCTET STRING raw }
  MarshalStd([][]byte) = SEQUENCE OF OCTET STRING          (used by rp/ipa.go:209)
"""


class DerError(ValueError):
    pass


def _len(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def tlv(tag, content):
    return bytes([tag]) + _len(len(content)) + content


def octet(b):
    return tlv(0x04, bytes(b))


def integer(v):
    n = max(1, (v.bit_length() + 8) // 8)  # two's complement, minimal
    b = v.to_bytes(n, "big", signed=True)
    while len(b) > 1 and ((b[0] == 0 and b[1] < 0x80) or (b[0] == 0xFF and b[1] >= 0x80)):
        b = b[1:]
    return tlv(0x02, b)


def seq(*items):
    return tlv(0x30, b"".join(items))


def marshal_std_bytes_list(items):
    """asn1.Marshal([][]byte{...})"""
    return seq(*[octet(x) for x in items])


def values(items):
    """asn1.Marshal(Values{items})"""
    return seq(seq(*[octet(x) for x in items]))


def element(curve_id, raw):
    return seq(integer(curve_id), octet(raw))


# ------------------------------------------------------------------ decode
def read_tlv(b, i=0):
    """-> (tag, content, next_index).  DER: definite, minimal lengths."""
    if i + 2 > len(b):
        raise DerError("truncated")
    tag = b[i]
    if tag & 0x1F == 0x1F:
        raise DerError("high tag")
    ln = b[i + 1]
    i += 2
    if ln & 0x80:
        nb = ln & 0x7F
        if nb == 0 or nb > 4 or i + nb > len(b):
            raise DerError("bad length")
        if b[i] == 0:
            raise DerError("non-minimal length")
        ln = int.from_bytes(b[i:i + nb], "big")
        i += nb
        if ln < 0x80:
            raise DerError("non-minimal length")
    if i + ln > len(b):
        raise DerError("truncated content")
    return tag, bytes(b[i:i + ln]), i + ln


def parse_seq_of_octets(content):
    out = []
    i = 0
    while i < len(content):
        tag, c, i = read_tlv(content, i)
        if tag != 0x04:
            raise DerError("expected OCTET STRING")
        out.append(c)
    return out


def unmarshal_values(b):
    """asn1.Unmarshal(b, &Values{}) -> list of bytes; trailing data ignored,
    extra struct fields ignored (Go semantics)."""
    tag, c, _ = read_tlv(b, 0)
    if tag != 0x30:
        raise DerError("expected SEQUENCE")
    if not c:
        raise DerError("sequence truncated")
    tag2, c2, _ = read_tlv(c, 0)
    if tag2 != 0x30:
        raise DerError("expected SEQUENCE OF")
    return parse_seq_of_octets(c2)


def unmarshal_bytes_list(b):
    tag, c, _ = read_tlv(b, 0)
    if tag != 0x30:
        raise DerError("expected SEQUENCE")
    return parse_seq_of_octets(c)


def unmarshal_element(b):
    """asn1.Unmarshal(b, &Element{}) with the 'no trailing bytes' rule of
    unmarshaller.Next (asn1.go:168-174)."""
    tag, c, nxt = read_tlv(b, 0)
    if tag != 0x30:
        raise DerError("expected SEQUENCE")
    if nxt != len(b):
        raise DerError("values should not have trailing bytes")
    t1, ci, j = read_tlv(c, 0)
    if t1 != 0x02 or not ci or len(ci) > 8:
        raise DerError("bad INTEGER")
    if len(ci) > 1 and ((ci[0] == 0 and ci[1] < 0x80) or (ci[0] == 0xFF and ci[1] >= 0x80)):
        raise DerError("integer not minimally-encoded")
    cid = int.from_bytes(ci, "big", signed=True)
    t2, raw, _ = read_tlv(c, j)
    if t2 != 0x04:
        raise DerError("expected OCTET STRING")
    return cid, raw


def unmarshal_values_strict(b):
    """asn1.Unmarshal(e.Raw, &Values{}) with 'no trailing bytes' (asn1.go:188-195)."""
    tag, c, nxt = read_tlv(b, 0)
    if nxt != len(b):
        raise DerError("values should not have trailing bytes")
    return unmarshal_values(b)
