"""fts_gpu — MI355X batch verifier for zkatdlog ("nogh" v1) token proofs.

Host-side mirror of the reference verifier API (paths relative to
token/core/zkatdlog/nogh/v1/crypto/ of fabric-token-sdk):

===========================================  =========================================
reference                                    here
===========================================  =========================================
``PublicParams.Deserialize`` setup.go:319     ``PublicParams(raw, bit_length, device)``
``rp.NewRangeVerifier(...).Verify``           ``RangeVerifier(pp, com).Verify(rp_bytes)``
  bulletproof.go:184-205,252-333
``rp.NewRangeCorrectnessVerifier.Verify``     ``RangeCorrectnessVerifier``
  rangecorrectness.go:118-162
``transfer.NewVerifier(in,out,pp).Verify``    ``TransferVerifier(in, out, pp).Verify(proof)``
  transfer/transfer.go:49-60,153-197
``issue.NewVerifier(tokens,pp).Verify``       ``IssueVerifier(tokens, pp).Verify(proof)``
  issue/verifier.go:24-57
gnark-crypto G1 ``MultiExp`` (config C3)      ``PublicParams.msm`` / :class:`StagedMsm`
===========================================  =========================================

``Verify`` returns ``None`` on success and raises :class:`VerifyError`
carrying the reference's error string otherwise.  The batch entry points
(``PublicParams.verify_range_proofs`` / ``verify_transfers`` /
``verify_issues`` and :class:`StagedRangeBatch`) are what a validator that
aggregates many actions calls; every one of them runs the HIP kernels of
``libfts_gpu.so`` — there is no CPU fallback.
"""
import ctypes as C

import numpy as np

from . import _lib as L
from ._lib import (FTS_OK, FTS_E_MALFORMED, FTS_E_RP_NIL, FTS_E_RP_INVALID, FTS_E_IPA_NIL, FTS_E_IPA_LEN,  # noqa
                   FTS_E_IPA_INVALID, FTS_E_RC_COUNT, FTS_E_TAS_INVALID, FTS_E_ST_INVALID, FTS_DEVICE_NONE,
                   FTS_E_ACTION_INVALID, FTS_E_OPEN_MISMATCH, FTS_SEED_OS_RANDOM, FtsError)
from . import request  # noqa: F401  (TokenRequest writers)


class VerifyError(Exception):
    """Verification failure; ``str(e)`` is the reference's error chain."""

    def __init__(self, msg, status, index=-1):
        super().__init__(msg)
        self.status = status
        self.index = index


def _rp_message(status):
    return L.status_str(status)


def transfer_message(status, index):
    """Error string of transfer.Verify (transfer.go:153-197) for a verdict."""
    if status == FTS_OK:
        return None
    if status == FTS_E_MALFORMED:
        return "invalid transfer proof: failed to deserialize proof"
    if status == FTS_E_TAS_INVALID:
        return "invalid transfer proof: invalid sum and type proof"
    if status == FTS_E_RC_COUNT:
        return "invalid range proof"
    return "invalid range proof at index %d: %s" % (index, _rp_message(status))


def issue_message(status, index):
    """Error string of issue.Verify (issue/verifier.go:32-57) for a verdict."""
    if status == FTS_OK:
        return None
    if status == FTS_E_MALFORMED:
        return "failed to deserialize proof"
    if status == FTS_E_ST_INVALID:
        return "invalid issue proof: invalid same type proof"
    if status == FTS_E_RC_COUNT:
        return "invalid issue proof: invalid range proof"
    return "invalid issue proof: invalid range proof at index %d: %s" % (index, _rp_message(status))


def inspect_request(raw):
    """host-only decode of one serialized TokenRequest (fts_request_inspect):
    dict(status, fail_action, n_issue, n_transfer, pre_status, pre_action)"""
    out = [C.c_int32() for _ in range(6)]
    L.check("fts_request_inspect", L.lib.fts_request_inspect(raw, len(raw), *[C.byref(o) for o in out]))
    keys = ("status", "fail_action", "n_issue", "n_transfer", "pre_status", "pre_action")
    return {k: o.value for k, o in zip(keys, out)}


def decode_metadata(raw):
    """host-only token.Metadata.Deserialize (fts_token_metadata_decode): None if it does
    not decode, else (type, value32 or None, bf32 or None) with value / bf mod r"""
    st, toff, tlen, has = C.c_int32(), C.c_size_t(), C.c_size_t(), C.c_int32()
    v, b = C.create_string_buffer(32), C.create_string_buffer(32)
    L.check("fts_token_metadata_decode", L.lib.fts_token_metadata_decode(
        raw, len(raw), C.byref(st), C.byref(toff), C.byref(tlen), v, b, C.byref(has)))
    if st.value != FTS_OK:
        return None
    return (raw[toff.value:toff.value + tlen.value], v.raw if has.value & 1 else None,
            b.raw if has.value & 2 else None)


def _ptr_array(blobs):
    bufs = [C.create_string_buffer(b, len(b)) if b else None for b in blobs]
    ptrs = (C.c_void_p * len(blobs))(*[C.cast(b, C.c_void_p) if b is not None else None for b in bufs])
    lens = (C.c_size_t * len(blobs))(*[len(b) for b in blobs])
    return bufs, ptrs, lens


class PublicParams:
    """A verification context: parsed public parameters plus their device
    tables (fixed-base windows of every generator) on one MI355X."""

    def __init__(self, raw, bit_length=None, device=0, devices=None, table_budget=None, wide_bits=None,
                 lanes=None):
        """device: one HIP ordinal (FTS_DEVICE_NONE: host-only); devices: a list of
        ordinals -> a multi-device context (fts_ctx_create_devices) whose batch calls
        shard over them and return verdicts in caller order.  table_budget (bytes) /
        wide_bits (20, 22) / lanes: fts_ctx_opts (fts_ctx_create_opts)"""
        self._ctx = C.c_void_p()
        if devices is None and (table_budget or wide_bits or lanes):
            o = L.CtxOpts(int(bit_length or 0), int(wide_bits or 0), int(table_budget or 0), int(lanes or 0), 0)
            rc = L.lib.fts_ctx_create_opts(raw, len(raw), int(device), C.byref(o), C.byref(self._ctx))
        elif devices is not None:
            arr = (C.c_int32 * len(devices))(*devices)
            rc = L.lib.fts_ctx_create_devices(raw, len(raw), int(bit_length or 0), arr, len(devices),
                                               C.byref(self._ctx))
        elif bit_length:
            rc = L.lib.fts_ctx_create_bits(raw, len(raw), int(bit_length), int(device), C.byref(self._ctx))
        else:
            rc = L.lib.fts_ctx_create(raw, len(raw), int(device), C.byref(self._ctx))
        L.check("fts_ctx_create", rc)
        info = L.PPInfo()
        L.check("fts_ctx_info", L.lib.fts_ctx_info(self._ctx, C.byref(info)))
        self.bit_length, self.rounds, self.device = info.bit_length, info.rounds, info.device
        self.max_token, self.table_bytes = info.max_token, info.table_bytes
        self.wide_bits, self.lanes = info.wide_bits, info.lanes
        devs = (C.c_int32 * 64)()
        self.devices = list(devs[:L.lib.fts_ctx_devices(self._ctx, devs, 64)])

    def close(self):
        if self._ctx:
            L.lib.fts_ctx_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def hold(self, n):
        """test hook (fts_debug_hold): no device pass starts until n calls are queued"""
        L.check("fts_debug_hold", L.lib.fts_debug_hold(self._ctx, int(n)))

    def dispatch_stats(self):
        """(passes, calls served, most calls in one pass, action calls) since creation"""
        out = (C.c_int64 * 4)()
        L.check("fts_debug_dispatch_stats", L.lib.fts_debug_dispatch_stats(self._ctx, out))
        return tuple(out)

    def reserve(self, max_pass_proofs=0):
        """pre-allocate every device lane for passes of up to max_pass_proofs
        (0: the coalescing cap) -- no allocation once batches flow"""
        L.check("fts_ctx_reserve", L.lib.fts_ctx_reserve(self._ctx, max_pass_proofs))

    # ------------------------------------------------------------ verify
    def verify_range_proofs(self, proofs, commitments):
        """Batch of standalone range proofs -> np.int32 verdicts."""
        n = len(proofs)
        assert len(commitments) == n
        bufs, ptrs, lens = _ptr_array(proofs)
        coms = b"".join(commitments)
        st = np.zeros(n, dtype=np.int32)
        L.check("fts_rp_verify_batch", L.lib.fts_rp_verify_batch(
            self._ctx, n, ptrs, lens, coms, st.ctypes.data_as(C.POINTER(C.c_int32))))
        return st

    def msm(self, points, scalars):
        """sum_i k_i P_i (fts_msm_g1): points = 64-byte X||Y BE each (or one
        joined bytes object), scalars = 32-byte BE each -> 64-byte result"""
        pts = points if isinstance(points, (bytes, bytearray)) else b"".join(points)
        scs = scalars if isinstance(scalars, (bytes, bytearray)) else b"".join(scalars)
        n = len(pts) // 64
        assert len(pts) == 64 * n and len(scs) == 32 * n
        out = C.create_string_buffer(64)
        L.check("fts_msm_g1", L.lib.fts_msm_g1(self._ctx, n, pts, scs, out))
        return out.raw

    def stage_msm(self, points, scalars):
        return StagedMsm(self, points, scalars)

    def stage_msm_multiples(self, ks, scalars):
        """n distinct points k_i * ped1 generated on the device (ks: 32-byte BE each)"""
        return StagedMsm(self, None, scalars, multiples=ks)

    def verify_transfers(self, transfers):
        """transfers: list of (inputs[list of 64B], outputs[list], proof bytes) ->
        (status, fail_index) arrays."""
        return self.prepare_transfers(transfers).verify()

    def verify_actions(self, transfers, issues):
        """mixed batch in one device pass -> (st_transfers, fail_transfers, st_issues, fail_issues)"""
        return self.prepare_actions(transfers, issues).verify()

    def prepare_actions(self, transfers, issues):
        return ActionBatch(self, transfers, issues)

    def prepare_transfers(self, transfers):
        """the fts_transfer_item array of a batch (host buffers the C-ABI borrows),
        reusable across verify() calls"""
        return TransferBatch(self, transfers)

    def verify_issues(self, issues):
        """issues: list of (tokens[list of 64B], proof bytes) -> (status, fail_index)."""
        n = len(issues)
        items = (L.IssueItem * n)()
        keep = []
        for i, (toks, proof) in enumerate(issues):
            bt = C.create_string_buffer(b"".join(toks) or b"\0")
            bp = C.create_string_buffer(proof or b"\0", max(1, len(proof)))
            keep += [bt, bp]
            items[i] = L.IssueItem(C.cast(bt, C.c_void_p), len(toks), C.cast(bp, C.c_void_p), len(proof))
        st = np.zeros(n, dtype=np.int32)
        fi = np.zeros(n, dtype=np.int32)
        L.check("fts_issue_verify_batch", L.lib.fts_issue_verify_batch(
            self._ctx, n, items, st.ctypes.data_as(C.POINTER(C.c_int32)), fi.ctypes.data_as(C.POINTER(C.c_int32))))
        return st, fi

    def verify_requests(self, requests):
        """serialized TokenRequests -> (status, fail_action, fail_index) arrays
        (fts_request_verify_batch: every action's proofs in one device pass)"""
        return self.prepare_requests(requests).verify()

    def prepare_requests(self, requests):
        """the request pointer / length arrays the C-ABI borrows, reusable across verify() calls"""
        return RequestBatch(self, requests)

    def stage_range_proofs(self, proofs, commitments):
        return StagedRangeBatch(self, proofs, commitments)

    def last_timings(self):
        """{kernel: ms} of the last range-proof run (device time per launch class)"""
        return {name: ms for name, (ms, _) in self.last_timings_ex().items()}

    def last_timings_ex(self):
        """{kernel: (ms, algorithmic u32 MADs)} of the last range-proof run"""
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        mads = (C.c_double * 64)()
        m = L.lib.fts_last_timings_ex(self._ctx, names, ms, mads, 64)
        out = {}
        for i in range(m):
            k = names[i].decode()
            o = out.get(k, (0.0, 0.0))
            out[k] = (o[0] + ms[i], o[1] + mads[i])
        return out

    # ------------------------------------------------------------- prove
    def prepare_openings(self, openings):
        """Pack token openings ``(com64, type, value32, bf32)`` (None = nil field)
        into the fts_token_opening array once; the result feeds check_openings."""
        return OpeningBatch(openings)

    def check_openings(self, openings):
        """Batched token opening checks (fts_token_open_batch): one verdict per
        token, FTS_OK iff HashToZr(type) ped0 + value ped1 + bf ped2 == com
        (auditor.go:226-238, token.go:69-83)."""
        ob = openings if isinstance(openings, OpeningBatch) else OpeningBatch(openings)
        st = np.zeros(ob.n, dtype=np.int32)
        L.check("fts_token_open_batch", L.lib.fts_token_open_batch(
            self._ctx, ob.n, ob.items, st.ctypes.data_as(C.POINTER(C.c_int32))))
        return st

    def check_metadata_openings(self, coms, metas):
        """fts_token_metadata_open_batch: token.Data (64 B each) + serialized
        driver.Metadata per output -> one verdict per output (auditor GetAuditInfoFor*
        + InspectOutput, auditor.go:285-400,226-238)."""
        n = len(coms)
        assert len(metas) == n
        bufs, ptrs, lens = _ptr_array(metas)
        st = np.zeros(n, dtype=np.int32)
        L.check("fts_token_metadata_open_batch", L.lib.fts_token_metadata_open_batch(
            self._ctx, n, b"".join(coms), ptrs, lens, st.ctypes.data_as(C.POINTER(C.c_int32))))
        return st

    def token_commit(self, ttype, value, bf32):
        out = C.create_string_buffer(64)
        L.check("fts_token_commit", L.lib.fts_token_commit(self._ctx, ttype, len(ttype), value, bf32, out))
        return out.raw

    def prove_range(self, value, bf32, seed):
        buf = C.create_string_buffer(1 << 14)
        ln = C.c_size_t()
        com = C.create_string_buffer(64)
        L.check("fts_rp_prove", L.lib.fts_rp_prove(self._ctx, value, bf32, seed, buf, len(buf), C.byref(ln), com))
        return buf.raw[:ln.value], com.raw

    def prove_range_batch(self, values, bfs, seed, threads=0):
        n = len(values)
        vals = (C.c_uint64 * n)(*values)
        cap = n * (1500 + 150 * self.rounds) + 4096
        out = C.create_string_buffer(cap)
        offs = (C.c_size_t * n)()
        lens = (C.c_size_t * n)()
        coms = C.create_string_buffer(64 * n)
        L.check("fts_rp_prove_batch", L.lib.fts_rp_prove_batch(
            self._ctx, n, vals, b"".join(bfs), seed, threads, out, cap, offs, lens, coms))
        raw, cr = out.raw, coms.raw
        return [raw[offs[i]:offs[i] + lens[i]] for i in range(n)], [cr[64 * i:64 * i + 64] for i in range(n)]

    def prove_range_batch_gpu(self, values, bfs, seed):
        """rangeProver.Prove for a batch on the device (fts_rp_prove_batch_gpu): the
        same proofs as prove_range_batch (proof i seeded with seed + i)."""
        n = len(values)
        vals = (C.c_uint64 * n)(*values)
        cap = n * (1500 + 150 * self.rounds) + 4096
        out = np.empty(cap, dtype=np.uint8)
        offs = (C.c_size_t * n)()
        lens = (C.c_size_t * n)()
        coms = np.empty(64 * n, dtype=np.uint8)
        L.check("fts_rp_prove_batch_gpu", L.lib.fts_rp_prove_batch_gpu(
            self._ctx, n, vals, b"".join(bfs), seed, out.ctypes.data, cap, offs, lens, coms.ctypes.data))
        raw, cr = out[:offs[n - 1] + lens[n - 1]].tobytes() if n else b"", coms.tobytes()
        return [raw[offs[i]:offs[i] + lens[i]] for i in range(n)], [cr[64 * i:64 * i + 64] for i in range(n)]

    def _prove_actions_gpu(self, fn, actions, seed):
        wb = actions if isinstance(actions, WitnessBatch) else WitnessBatch(actions, self.rounds)
        n = wb.n
        out = np.empty(wb.cap, dtype=np.uint8)
        offs, lens = (C.c_size_t * n)(), (C.c_size_t * n)()
        L.check(fn, getattr(L.lib, fn)(self._ctx, n, wb.items, seed, out.ctypes.data, wb.cap, offs, lens))
        raw = out[:offs[n - 1] + lens[n - 1]].tobytes() if n else b""
        return [raw[offs[i]:offs[i] + lens[i]] for i in range(n)]

    def prove_transfers_gpu(self, transfers, seed):
        """transfer.NewProver(...).Prove() for a batch on the device
        (fts_transfer_prove_batch_gpu): transfers = [(type, in_values, in_bfs,
        out_values, out_bfs)], transfer i seeded with seed + i -- the proofs of
        prove_transfer."""
        return self._prove_actions_gpu("fts_transfer_prove_batch_gpu", transfers, seed)

    def prove_issues_gpu(self, issues, seed):
        """issue.NewProver(...).Prove() for a batch on the device: issues = [(type,
        values, bfs)], issue i seeded with seed + i -- the proofs of prove_issue."""
        if not isinstance(issues, WitnessBatch):
            issues = WitnessBatch([(t, [], [], v, b) for t, v, b in issues], self.rounds)
        return self._prove_actions_gpu("fts_issue_prove_batch_gpu", issues, seed)

    def prove_transfer(self, ttype, in_values, in_bfs, out_values, out_bfs, seed):
        buf = C.create_string_buffer(1 << 16)
        ln = C.c_size_t()
        iv = (C.c_uint64 * len(in_values))(*in_values)
        ov = (C.c_uint64 * len(out_values))(*out_values)
        L.check("fts_transfer_prove", L.lib.fts_transfer_prove(
            self._ctx, ttype, len(ttype), len(in_values), iv, b"".join(in_bfs), len(out_values), ov,
            b"".join(out_bfs), seed, buf, len(buf), C.byref(ln)))
        return buf.raw[:ln.value]

    def prove_issue(self, ttype, values, bfs, seed):
        buf = C.create_string_buffer(1 << 17)
        ln = C.c_size_t()
        v = (C.c_uint64 * len(values))(*values)
        L.check("fts_issue_prove", L.lib.fts_issue_prove(
            self._ctx, ttype, len(ttype), len(values), v, b"".join(bfs), seed, buf, len(buf), C.byref(ln)))
        return buf.raw[:ln.value]


class StagedRangeBatch:
    """Range proofs parsed and resident in HBM; ``verify()`` runs only the
    GPU verification (fts_rp_batch_verify)."""

    def __init__(self, pp, proofs, commitments):
        self.pp = pp
        self.n = len(proofs)
        self._b = C.c_void_p()
        bufs, ptrs, lens = _ptr_array(proofs)
        L.check("fts_rp_batch_stage", L.lib.fts_rp_batch_stage(
            pp._ctx, self.n, ptrs, lens, b"".join(commitments), C.byref(self._b)))

    def verify(self, want_status=True):
        st = np.zeros(self.n, dtype=np.int32) if want_status else None
        L.check("fts_rp_batch_verify", L.lib.fts_rp_batch_verify(
            self.pp._ctx, self._b, st.ctypes.data_as(C.POINTER(C.c_int32)) if want_status else None))
        return st

    def merged(self):
        """staged batches in the device pass that verified this one last (coalescing)"""
        return int(L.lib.fts_rp_batch_merged(self._b))

    def timings(self):
        """{kernel: (ms, algorithmic u32 MADs)} of this batch's last verify()"""
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        mads = (C.c_double * 64)()
        m = L.lib.fts_rp_batch_timings(self._b, names, ms, mads, 64)
        out = {}
        for i in range(m):
            k = names[i].decode()
            o = out.get(k, (0.0, 0.0))
            out[k] = (o[0] + ms[i], o[1] + mads[i])
        return out

    def close(self):
        if self._b:
            L.lib.fts_rp_batch_free(self._b)
            self._b = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------ reference-shaped verifiers
class TransferBatch:
    """Host-side fts_transfer_item array (what the Go shim hands over per batch)."""

    def __init__(self, pp, transfers):
        self.pp = pp
        self.n = len(transfers)
        self.items = (L.TransferItem * max(1, self.n))()
        self._keep = []
        for i, (ins, outs, proof) in enumerate(transfers):
            bi = C.create_string_buffer(b"".join(ins) or b"\0")
            bo = C.create_string_buffer(b"".join(outs) or b"\0")
            bp = C.create_string_buffer(proof or b"\0", max(1, len(proof)))
            self._keep += [bi, bo, bp]
            self.items[i] = L.TransferItem(C.cast(bi, C.c_void_p), len(ins), C.cast(bo, C.c_void_p), len(outs),
                                           C.cast(bp, C.c_void_p), len(proof))

    def verify(self):
        st = np.zeros(self.n, dtype=np.int32)
        fi = np.zeros(self.n, dtype=np.int32)
        L.check("fts_transfer_verify_batch", L.lib.fts_transfer_verify_batch(
            self.pp._ctx, self.n, self.items, st.ctypes.data_as(C.POINTER(C.c_int32)),
            fi.ctypes.data_as(C.POINTER(C.c_int32))))
        return st, fi


class RequestBatch:
    """Serialized TokenRequests as the host hands them over (pointer + length per request)."""

    def __init__(self, pp, requests):
        self.pp = pp
        self.n = len(requests)
        self._keep, self.ptrs, self.lens = _ptr_array(requests)

    def verify(self):
        st = np.zeros(self.n, dtype=np.int32)
        fa = np.zeros(self.n, dtype=np.int32)
        fi = np.zeros(self.n, dtype=np.int32)
        I32 = C.POINTER(C.c_int32)
        L.check("fts_request_verify_batch", L.lib.fts_request_verify_batch(
            self.pp._ctx, self.n, self.ptrs, self.lens, st.ctypes.data_as(I32), fa.ctypes.data_as(I32),
            fi.ctypes.data_as(I32)))
        return st, fa, fi


class IssueBatch:
    """Host-side fts_issue_item array."""

    def __init__(self, pp, issues):
        self.pp = pp
        self.n = len(issues)
        self.items = (L.IssueItem * max(1, self.n))()
        self._keep = []
        for i, (toks, proof) in enumerate(issues):
            bt = C.create_string_buffer(b"".join(toks) or b"\0")
            bp = C.create_string_buffer(proof or b"\0", max(1, len(proof)))
            self._keep += [bt, bp]
            self.items[i] = L.IssueItem(C.cast(bt, C.c_void_p), len(toks), C.cast(bp, C.c_void_p), len(proof))


class ActionBatch:
    """Transfers + issues verified together (fts_actions_verify_batch)."""

    def __init__(self, pp, transfers, issues):
        self.pp = pp
        self.tr = TransferBatch(pp, transfers)
        self.iss = IssueBatch(pp, issues)

    def verify(self):
        nt, ni = self.tr.n, self.iss.n
        st_t, fi_t = np.zeros(max(1, nt), dtype=np.int32), np.zeros(max(1, nt), dtype=np.int32)
        st_i, fi_i = np.zeros(max(1, ni), dtype=np.int32), np.zeros(max(1, ni), dtype=np.int32)
        ptr = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
        L.check("fts_actions_verify_batch", L.lib.fts_actions_verify_batch(
            self.pp._ctx, nt, self.tr.items, ni, self.iss.items, ptr(st_t), ptr(fi_t), ptr(st_i), ptr(fi_i)))
        return st_t[:nt], fi_t[:nt], st_i[:ni], fi_i[:ni]


class StagedMsm:
    """MSM inputs validated and resident in HBM; ``run()`` is the device MSM only."""

    def __init__(self, pp, points, scalars, multiples=None):
        """points: n x 64-byte X||Y BE; or, with multiples = n x 32-byte BE k_i and
        points None, the distinct points k_i * ped1 generated on the device
        (fts_msm_stage_multiples, config C3 at scale)"""
        self.pp = pp
        scs = scalars if isinstance(scalars, (bytes, bytearray)) else b"".join(scalars)
        self._b = C.c_void_p()
        if multiples is not None:
            ks = multiples if isinstance(multiples, (bytes, bytearray)) else b"".join(multiples)
            self.n = len(ks) // 32
            L.check("fts_msm_stage_multiples",
                    L.lib.fts_msm_stage_multiples(pp._ctx, self.n, ks, scs, C.byref(self._b)))
            return
        pts = points if isinstance(points, (bytes, bytearray)) else b"".join(points)
        self.n = len(pts) // 64
        L.check("fts_msm_stage", L.lib.fts_msm_stage(pp._ctx, self.n, pts, scs, C.byref(self._b)))

    def run(self):
        out = C.create_string_buffer(64)
        L.check("fts_msm_run", L.lib.fts_msm_run(self.pp._ctx, self._b, out))
        return out.raw

    def points(self, lo=0, count=None):
        """the staged points [lo, lo + count) as 64-byte X||Y BE (fts_msm_points)"""
        count = self.n - lo if count is None else count
        out = C.create_string_buffer(64 * max(1, count))
        L.check("fts_msm_points", L.lib.fts_msm_points(self.pp._ctx, self._b, lo, count, out))
        return out.raw[:64 * count]

    def timings(self):
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        mads = (C.c_double * 64)()
        m = L.lib.fts_msm_timings(self._b, names, ms, mads, 64)
        out = {}
        for i in range(m):
            k = names[i].decode()
            o = out.get(k, (0.0, 0.0))
            out[k] = (o[0] + ms[i], o[1] + mads[i])
        return out

    def close(self):
        if self._b:
            L.lib.fts_msm_free(self._b)
            self._b = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OpeningBatch:
    """fts_token_opening[] over contiguous buffers (kept alive with the batch)."""

    def __init__(self, openings):
        n = self.n = len(openings)
        fixed = [(64, 0), (32, 2), (32, 3)]
        self._blobs = []
        cols = np.zeros((n, 5), dtype=np.uint64)
        for size, k in fixed:
            vals = [o[k] for o in openings]
            for v in vals:
                assert v is None or len(v) == size
            blob = np.frombuffer(b"".join(v if v is not None else bytes(size) for v in vals) or b"\0", dtype=np.uint8)
            self._blobs.append(blob)
            col = {0: 0, 2: 3, 3: 4}[k]
            cols[:, col] = blob.ctypes.data + np.arange(n, dtype=np.uint64) * size
            nil = np.array([v is None for v in vals], dtype=bool)
            cols[nil, col] = 0
        types = [o[1] or b"" for o in openings]
        tblob = np.frombuffer(b"".join(types) or b"\0", dtype=np.uint8)
        self._blobs.append(tblob)
        lens = np.array([len(t) for t in types], dtype=np.uint64)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if n else lens
        cols[:, 1] = tblob.ctypes.data + offs
        cols[:, 2] = lens
        self._cols = np.ascontiguousarray(cols)
        self.items = self._cols.ctypes.data_as(C.POINTER(L.TokenOpening))


class WitnessBatch:
    """fts_action_witness[] over contiguous buffers: actions = [(type, in_values,
    in_bfs, out_values, out_bfs)] (issues: empty inputs); reusable across calls."""

    def __init__(self, actions, rounds=6):
        n = self.n = len(actions)
        cols = np.zeros((n, 8), dtype=np.uint64)
        self._keep = []

        def blob(parts, col_ptr, col_len=None, unit=1):
            data = b"".join(parts)
            arr = np.frombuffer(data or b"\0", dtype=np.uint8)
            self._keep.append(arr)
            lens = np.array([len(p) for p in parts], dtype=np.uint64)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if n else lens
            cols[:, col_ptr] = arr.ctypes.data + offs
            if col_len is not None:
                cols[:, col_len] = lens // unit

        u64 = lambda vs: np.asarray(vs, dtype=np.uint64).tobytes()  # noqa: E731
        blob([a[0] for a in actions], 0, 1)
        blob([u64(a[1]) for a in actions], 3, 2, 8)
        blob([b"".join(a[2]) for a in actions], 4)
        blob([u64(a[3]) for a in actions], 6, 5, 8)
        blob([b"".join(a[4]) for a in actions], 7)
        self.cap = 4096 + sum(1024 + 200 * len(a[1]) + len(a[3]) * (1500 + 150 * rounds) for a in actions)
        self._cols = np.ascontiguousarray(cols)
        self.items = self._cols.ctypes.data_as(C.POINTER(L.ActionWitness))


class Auditor:
    """The opening checks of audit.Auditor (crypto/audit/auditor.go): every
    output of every action is re-committed on the device in one batch; the
    error chain is the reference's (CheckIssueRequests / CheckTransferRequests
    :168-210, InspectOutputs :213-222, InspectOutput :226-238).  Identity
    inspection (InspectIdentity) is out of scope."""

    def __init__(self, pp):
        self.pp = pp

    def InspectOutputs(self, tokens):
        st = self.pp.check_openings(tokens)
        for i, s in enumerate(st):
            if s != FTS_OK:
                raise VerifyError(_inspect_message(int(s), i), int(s), i)

    def check_actions(self, actions, txid, kind="transfer"):
        """actions: list (one per action) of lists of openings; raises the error of
        the first failing output of the first failing action (auditor.go:178-210)."""
        flat = [t for a in actions for t in a]
        st = self.pp.check_openings(flat)
        pos = 0
        for k, a in enumerate(actions):
            for i in range(len(a)):
                s = int(st[pos + i])
                if s != FTS_OK:
                    what = "%d th transfer" % k if kind == "transfer" else "%d th issue" % k
                    raise VerifyError("audit of %s in tx [%s] failed: %s" % (what, txid, _inspect_message(s, i)), s, i)
            pos += len(a)


def _inspect_message(status, i):
    if status == FTS_E_OPEN_MISMATCH:
        return "failed inspecting output [%d]: output at index [%d] does not match the provided opening" % (i, i)
    return "failed inspecting output [%d]: invalid output at index [%d]" % (i, i)


class RangeVerifier:
    """rp.NewRangeVerifier(com, ...) / Verify (bulletproof.go:184-205,252-333).
    The generators come from ``pp`` exactly as RangeCorrectnessVerifier passes
    them (PedersenGenerators[1:], Left/Right, P, Q)."""

    def __init__(self, pp, commitment):
        self.pp, self.commitment = pp, commitment

    def Verify(self, rp_bytes):
        s = int(self.pp.verify_range_proofs([rp_bytes], [self.commitment])[0])
        if s != FTS_OK:
            raise VerifyError(_rp_message(s), s)


class TransferVerifier:
    """transfer.NewVerifier(inputs, outputs, pp) / Verify (transfer.go:49-60,153-197)."""

    def __init__(self, inputs, outputs, pp):
        self.inputs, self.outputs, self.pp = list(inputs), list(outputs), pp

    def Verify(self, proof):
        st, fi = self.pp.verify_transfers([(self.inputs, self.outputs, proof)])
        msg = transfer_message(int(st[0]), int(fi[0]))
        if msg:
            raise VerifyError(msg, int(st[0]), int(fi[0]))


class IssueVerifier:
    """issue.NewVerifier(tokens, pp) / Verify (issue/verifier.go:24-57)."""

    def __init__(self, tokens, pp):
        self.tokens, self.pp = list(tokens), pp

    def Verify(self, proof):
        st, fi = self.pp.verify_issues([(self.tokens, proof)])
        msg = issue_message(int(st[0]), int(fi[0]))
        if msg:
            raise VerifyError(msg, int(st[0]), int(fi[0]))
