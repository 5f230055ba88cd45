"""TokenRequest wire format (the bytes fts_request_verify_batch ingests).

Writers for the protobuf messages the reference serialises on the way to
Validator.VerifyTokenRequestFromRaw:

  TokenRequest{version=1, actions=2 Action{type=1, raw=2}, signatures=3,
               auditor_signatures=4}          driver/protos/request.proto:85-100,
                                              driver/request.go:38-66 (ToProtos/Bytes)
  TransferAction / IssueAction                nogh/protos/noghactions.proto,
                                              crypto/transfer/action.go:286-324 (Serialize),
                                              crypto/issue/action.go:191-229
  G1{raw = mathlib JSON {"curve":1,"element":base64(64 B)}}
                                              nogh/protos-go/utils/proto.go:22-31

Fields are written in field-number order, as proto.Marshal does; a `None`
sub-message is omitted (a nil pointer in Go).  Host-side plumbing for callers
and tests -- nothing here verifies anything.
"""
import base64

ISSUE = 0      # request.proto ActionType
TRANSFER = 1


def varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def field_varint(no, v):
    return varint(no << 3) + varint(v)


def field_bytes(no, b):
    return varint((no << 3) | 2) + varint(len(b)) + bytes(b)


def msg(no, body):
    """singular / repeated message field; body None -> omitted (nil)"""
    return b"" if body is None else field_bytes(no, body)


def opt_bytes(no, b):
    """proto3 bytes/string: empty values are not written"""
    if isinstance(b, str):
        b = b.encode()
    return field_bytes(no, b) if b else b""


def g1_json(point64):
    """mathlib G1.MarshalJSON of a 64-byte uncompressed BN254 point"""
    return b'{"curve":1,"element":"' + base64.b64encode(bytes(point64)) + b'"}'


def g1(point64):
    """nogh.G1 message (None -> nil pointer; b"" -> G1 with empty raw)"""
    if point64 is None:
        return None
    return opt_bytes(1, g1_json(point64) if len(point64) else b"")


def token(owner, data64):
    """nogh.Token{owner=1, data=2 G1}"""
    return opt_bytes(1, owner) + msg(2, g1(data64))


def token_id(tx_id, index=0):
    return opt_bytes(1, tx_id) + (field_varint(2, index) if index else b"")


def _metadata(no, md):
    out = b""
    for k, v in sorted((md or {}).items()):
        out += field_bytes(no, opt_bytes(1, k) + opt_bytes(2, v))
    return out


def transfer_action(inputs, outputs, proof, metadata=None):
    """inputs: [(tx_id, index, owner, commitment64)] (or a raw TransferActionInput body);
    outputs: [(owner, commitment64)] (or None for a nil output token)"""
    out = b""
    for x in inputs:
        if isinstance(x, (bytes, bytearray)):
            out += field_bytes(1, x)
            continue
        tx, idx, owner, com = x
        out += field_bytes(1, msg(1, token_id(tx, idx)) + msg(2, token(owner, com)))
    for o in outputs:
        out += field_bytes(2, b"" if o is None else msg(1, token(o[0], o[1])))
    if proof is not None:
        out += field_bytes(3, opt_bytes(1, proof))
    return out + _metadata(4, metadata)


def issue_action(issuer, outputs, proof, inputs=(), metadata=None):
    """outputs: [(owner, commitment64)] (None: nil output); inputs: [(tx_id, index, token bytes)]"""
    out = msg(1, None if issuer is None else opt_bytes(1, issuer))
    for tx, idx, tok in inputs:
        out += field_bytes(2, msg(1, token_id(tx, idx)) + opt_bytes(2, tok))
    for o in outputs:
        out += field_bytes(3, b"" if o is None else msg(1, token(o[0], o[1])))
    if proof is not None:
        out += field_bytes(4, opt_bytes(1, proof))
    return out + _metadata(5, metadata)


def token_request(actions, signatures=(), auditor_signatures=(), version=1):
    """actions: [(ISSUE|TRANSFER, raw action bytes)] in request order"""
    out = field_varint(1, version) if version else b""
    for typ, raw in actions:
        out += field_bytes(2, (field_varint(1, typ) if typ else b"") + opt_bytes(2, raw))
    for s in signatures:
        out += field_bytes(3, opt_bytes(1, s))
    for s in auditor_signatures:
        out += field_bytes(4, opt_bytes(1, s))
    return out


# ----------------------------------------------------------- token metadata
def zr_json(b32):
    """mathlib Zr.MarshalJSON: {"curve":1,"element":b64(Zr.Bytes())}"""
    return b'{"curve":1,"element":"' + base64.b64encode(b32) + b'"}'


def zr(b32):
    return field_bytes(1, zr_json(b32))


def der_tlv(tag, body):
    n = len(body)
    if n < 0x80:
        ln = bytes([n])
    else:
        nb = (n.bit_length() + 7) // 8
        ln = bytes([0x80 | nb]) + n.to_bytes(nb, "big")
    return bytes([tag]) + ln + body


def typed_token(typ, raw):
    """asn1.Marshal(TypedToken{Type, Token}) (services/tokens/typed.go:24-26)"""
    ib = typ.to_bytes(max(1, (typ.bit_length() + 8) // 8), "big", signed=True)
    return der_tlv(0x30, der_tlv(0x02, ib) + der_tlv(0x04, raw))


def token_metadata(ttype, value32, bf32, issuer=b"", typ=2):
    """token.Metadata.Serialize (crypto/token/token.go:160-180): TypedToken-wrapped
    TokenMetadata{type, value, blinding_factor, issuer}; value32 / bf32 None = nil Zr"""
    body = field_bytes(1, ttype) if ttype else b""
    if value32 is not None:
        body += msg(2, zr(value32))
    if bf32 is not None:
        body += msg(3, zr(bf32))
    body += msg(4, field_bytes(1, issuer) if issuer else b"")
    return typed_token(typ, body)
