"""Host-only TokenRequest ingest (fts_request_inspect, no device): the
deserialisation and structural verdicts of VerifyTokenRequestFromRaw that
precede the ZK proofs.

  TokenRequest.FromBytes / FromProtos     driver/request.go:46-95
  DeserializeActions (issues, transfers)  nogh/v1/validator/validator.go:27-47
  transfer Action.Deserialize / Validate  crypto/transfer/action.go:76-111,244-283,326-362
  issue Action.Deserialize / Validate     crypto/issue/action.go:38-45,161-185,231-282
  FromG1Proto / FromZrProto               nogh/protos-go/utils/proto.go:39-72

The requests are written with fts_gpu.request (the reference's proto layout);
protobuf-go semantics exercised: unknown fields and wire-type mismatches are
skipped, singular messages merge, proto3 strings must be UTF-8, enum values are
int32-truncated.  No serialized TokenRequest fixture ships with the reference,
so the expected verdicts follow its code paths (cited per case)."""
import json
import os

import pytest

from conftest import GOLDEN

F = pytest.importorskip("fts_gpu")
R = F.request

with open(os.path.join(GOLDEN, "transfer_golden.json")) as _f:
    _T = json.load(_f)[0]
IN = [bytes.fromhex(h) for h in _T["inputs"]]
OUT = [bytes.fromhex(h) for h in _T["outputs"]]
PROOF = bytes.fromhex(_T["proof"])

OK, MAL, INV = F.FTS_OK, F.FTS_E_MALFORMED, F.FTS_E_ACTION_INVALID


def tr(inputs=None, outputs=None, proof=PROOF, **kw):
    inputs = [("tx%d" % i, i, b"alice", c) for i, c in enumerate(IN)] if inputs is None else inputs
    outputs = [(b"bob", c) for c in OUT] if outputs is None else outputs
    return R.transfer_action(inputs, outputs, proof, **kw)


def iss(issuer=b"issuer", outputs=None, proof=b"\x30\x00", **kw):
    outputs = [(b"bob", c) for c in OUT] if outputs is None else outputs
    return R.issue_action(issuer, outputs, proof, **kw)


def req(*actions, sigs=(b"sig",), **kw):
    return R.token_request(list(actions), sigs, **kw)


def inspect(raw):
    r = F.inspect_request(raw)
    return r["status"], r["fail_action"], r["pre_status"], r["pre_action"]


def g1_raw_msg(raw_json):
    return R.opt_bytes(1, raw_json)


def test_honest_counts():
    r = F.inspect_request(req((R.ISSUE, iss()), (R.TRANSFER, tr()), (R.TRANSFER, tr())))
    assert r == dict(status=OK, fail_action=-1, n_issue=1, n_transfer=2, pre_status=OK, pre_action=-1)


def test_request_level_malformed():
    assert inspect(b"") == (MAL, -1, OK, -1)                       # "empty token request"
    assert inspect(b"\x12\x05ab") == (MAL, -1, OK, -1)             # truncated length-delimited field
    assert inspect(b"\x12") == (MAL, -1, OK, -1)                   # truncated varint
    assert inspect(b"\x02\x00") == (MAL, -1, OK, -1)               # field number 0
    assert inspect(b"\x0b") == (MAL, -1, OK, -1)                   # group wire type
    assert inspect(R.field_bytes(2, b"\x12\x03xy")) == (MAL, -1, OK, -1)  # Action message truncated
    assert inspect(R.field_bytes(3, b"\xff")) == (MAL, -1, OK, -1)       # Signature message truncated


def test_unknown_fields_and_wire_mismatch_skipped():
    base = req((R.TRANSFER, tr()))
    assert inspect(base + R.field_varint(9, 7) + R.field_bytes(15, b"zz")) == (OK, -1, OK, -1)
    # `actions` sent as a varint: an unknown field for protobuf-go -> request with no actions
    r = F.inspect_request(R.field_varint(2, 1))
    assert (r["status"], r["n_issue"], r["n_transfer"]) == (OK, 0, 0)
    assert inspect(R.token_request([])) == (OK, -1, OK, -1)        # version only: nothing to verify


def test_action_types():
    assert inspect(req((R.TRANSFER, tr()), (2, tr()))) == (MAL, 1, OK, -1)   # request.go:78-79
    # ActionType is an int32 enum: 2^32 + 1 truncates to TRANSFER
    act = R.field_bytes(2, R.field_varint(1, (1 << 32) + 1) + R.opt_bytes(2, tr()))
    r = F.inspect_request(act)
    assert (r["status"], r["n_transfer"]) == (OK, 1)
    # FromProtos checks every action type before any signature (request.go:69-93)
    assert inspect(req((R.TRANSFER, tr()), (7, b""), sigs=(b"",))) == (MAL, 1, OK, -1)


def test_signatures():
    assert inspect(req((R.TRANSFER, tr()), sigs=(b"",))) == (MAL, -1, OK, -1)          # "nil signature found"
    assert inspect(R.token_request([(R.TRANSFER, tr())], [b"s"], [b""])) == (MAL, -1, OK, -1)
    assert inspect(req((R.TRANSFER, tr()), sigs=())) == (OK, -1, OK, -1)


def test_action_deserialisation_order():
    bad = b"\x0a\x09"  # truncated TransferActionInput
    # DeserializeActions decodes every issue before any transfer (validator.go:29-45)
    assert inspect(req((R.TRANSFER, bad), (R.ISSUE, b"\x1a\x05"))) == (MAL, 1, OK, -1)
    assert inspect(req((R.TRANSFER, tr()), (R.TRANSFER, bad), (R.ISSUE, iss()))) == (MAL, 1, OK, -1)


@pytest.mark.parametrize("raw_json", [
    b'{"curve":1,"element":"' + __import__("base64").b64encode(b"\x01" + b"\x00" * 63) + b'"}',  # off curve
    b'{"curve":2,"element":"' + __import__("base64").b64encode(IN[0]) + b'"}',                  # other curve
    b'{"curve":1,"element":"***"}',                                                              # not base64
    b'{"curve":1,"element":"' + __import__("base64").b64encode(IN[0][:32]) + b'"}',             # short
])
def test_bad_g1_is_malformed(raw_json):
    bad_tok = R.opt_bytes(1, b"alice") + R.field_bytes(2, g1_raw_msg(raw_json))
    bad_in = R.msg(1, R.token_id("tx", 0)) + R.msg(2, bad_tok)
    assert inspect(req((R.TRANSFER, R.transfer_action([bad_in], [(b"b", OUT[0])], PROOF)))) == (MAL, 0, OK, -1)
    out = R.field_bytes(3, R.msg(1, bad_tok))
    assert inspect(req((R.ISSUE, R.msg(1, R.opt_bytes(1, b"i")) + out))) == (MAL, 0, OK, -1)


def test_nil_commitments():
    # empty G1 raw -> nil point (proto.go:40-42); transfer Token.Validate rejects it (token.go:89-91)
    assert inspect(req((R.TRANSFER, tr(outputs=[(b"bob", b"")])))) == (OK, -1, INV, 0)
    assert inspect(req((R.TRANSFER, tr(inputs=[("tx", 0, b"a", None)])))) == (OK, -1, INV, 0)
    # issue: Validate passes, the nil commitment reaches the verifier (a panic in the reference)
    assert inspect(req((R.ISSUE, iss(outputs=[(b"bob", b"")])))) == (OK, -1, MAL, 0)
    # nil output messages
    assert inspect(req((R.TRANSFER, tr(outputs=[None])))) == (OK, -1, INV, 0)
    assert inspect(req((R.ISSUE, iss(outputs=[(b"bob", OUT[0]), None])))) == (OK, -1, INV, 0)


def test_transfer_validate():
    # transfer/action.go:244-283
    assert inspect(req((R.TRANSFER, tr(inputs=[])))) == (OK, -1, INV, 0)                      # no inputs
    assert inspect(req((R.TRANSFER, tr(outputs=[])))) == (OK, -1, INV, 0)                     # no outputs
    assert inspect(req((R.TRANSFER, tr(inputs=[("", 0, b"a", IN[0])])))) == (OK, -1, INV, 0)  # empty tx id
    assert inspect(req((R.TRANSFER, tr(inputs=[("tx", 0, b"", IN[0])])))) == (OK, -1, INV, 0)  # no owner
    no_id = R.msg(2, R.token(b"a", IN[0]))
    assert inspect(req((R.TRANSFER, tr(inputs=[no_id])))) == (OK, -1, INV, 0)                 # nil ID
    no_tok = R.msg(1, R.token_id("tx", 0))
    assert inspect(req((R.TRANSFER, tr(inputs=[no_tok])))) == (OK, -1, INV, 0)                # nil token
    # redeem: outputs need no owner (Validate(false))
    assert inspect(req((R.TRANSFER, tr(outputs=[(b"", OUT[0])])))) == (OK, -1, OK, -1)


def test_issue_validate():
    # issue/action.go:161-185
    assert inspect(req((R.ISSUE, iss(issuer=None)))) == (OK, -1, INV, 0)
    assert inspect(req((R.ISSUE, iss(issuer=b"")))) == (OK, -1, INV, 0)
    assert inspect(req((R.ISSUE, iss(outputs=[])))) == (OK, -1, INV, 0)
    assert inspect(req((R.ISSUE, iss(inputs=[("tx", 0, b"")])))) == (OK, -1, INV, 0)
    assert inspect(req((R.ISSUE, iss(inputs=[("", 0, b"tok")])))) == (OK, -1, INV, 0)
    assert inspect(req((R.ISSUE, iss(inputs=[("tx", 3, b"tok")])))) == (OK, -1, OK, -1)


def test_pre_verdict_reference_order():
    # issues are verified before transfers: the issue at index 1 is reported first
    r = req((R.TRANSFER, tr(inputs=[])), (R.ISSUE, iss(issuer=None)))
    assert inspect(r) == (OK, -1, INV, 1)


def test_utf8_strings():
    good = [("tx-é中\U0001F600", 0, b"a", IN[0])]
    assert inspect(req((R.TRANSFER, tr(inputs=good)))) == (OK, -1, OK, -1)
    for bad in (b"\xff", b"\xc0\xaf", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xe4\xb8"):
        tid = R.field_bytes(1, b"tx" + bad)
        inp = R.msg(1, tid) + R.msg(2, R.token(b"a", IN[0]))
        assert inspect(req((R.TRANSFER, tr(inputs=[inp])))) == (MAL, 0, OK, -1), bad
        assert inspect(req((R.TRANSFER, tr(metadata={b"k" + bad: b"v"})))) == (MAL, 0, OK, -1), bad
    assert inspect(req((R.TRANSFER, tr(metadata={"key": b"\xff\xfe"})))) == (OK, -1, OK, -1)  # bytes values


def test_singular_message_merge():
    import base64
    bad = g1_raw_msg(b'{"curve":1,"element":"***"}')
    good = g1_raw_msg(R.g1_json(IN[0]))
    # Token.data twice: the G1 messages merge, the last raw wins
    tok = R.opt_bytes(1, b"alice") + R.field_bytes(2, bad) + R.field_bytes(2, good)
    inp = R.msg(1, R.token_id("tx", 0)) + R.msg(2, tok)
    assert inspect(req((R.TRANSFER, tr(inputs=[inp])))) == (OK, -1, OK, -1)
    tok2 = R.opt_bytes(1, b"alice") + R.field_bytes(2, good) + R.field_bytes(2, bad)
    inp2 = R.msg(1, R.token_id("tx", 0)) + R.msg(2, tok2)
    assert inspect(req((R.TRANSFER, tr(inputs=[inp2])))) == (MAL, 0, OK, -1)
    # TokenID split across two occurrences: index from one, id from the other
    inp3 = R.msg(1, R.field_varint(2, 4)) + R.msg(1, R.opt_bytes(1, "tx")) + R.msg(2, R.token(b"a", IN[0]))
    assert inspect(req((R.TRANSFER, tr(inputs=[inp3])))) == (OK, -1, OK, -1)
    del base64


def test_upgrade_witness_decoding():
    zr_good = R.opt_bytes(1, b'{"curve":1,"element":"AQI="}')
    fab = R.opt_bytes(1, b"o") + R.opt_bytes(2, "USD") + R.opt_bytes(3, "0x10")
    wit = R.msg(1, fab) + R.msg(2, zr_good)
    inp = R.msg(1, R.token_id("tx", 0)) + R.msg(2, R.token(b"a", IN[0])) + R.msg(3, wit)
    assert inspect(req((R.TRANSFER, tr(inputs=[inp])))) == (OK, -1, OK, -1)
    # a present Zr with empty raw fails Zr.UnmarshalJSON (proto.go:62-70)
    wit_bad = R.msg(1, fab) + R.msg(2, b"")
    inp_bad = R.msg(1, R.token_id("tx", 0)) + R.msg(2, R.token(b"a", IN[0])) + R.msg(3, wit_bad)
    assert inspect(req((R.TRANSFER, tr(inputs=[inp_bad])))) == (MAL, 0, OK, -1)
    fab_bad = R.opt_bytes(2, b"\xff")
    inp_bad2 = R.msg(1, R.token_id("tx", 0)) + R.msg(2, R.token(b"a", IN[0])) + R.msg(3, R.msg(1, fab_bad))
    assert inspect(req((R.TRANSFER, tr(inputs=[inp_bad2])))) == (MAL, 0, OK, -1)
