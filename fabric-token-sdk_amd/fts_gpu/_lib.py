"""ctypes binding of libfts_gpu.so (include/fts_gpu.h).

The shared library is built in-tree by ``make -C fabric-token-sdk_amd`` (see
``__graft_entry__.build``).  There is no fallback: if the library is missing
or fails to load, importing this module raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FTS_LIB: alternative in-tree build of the same library (A/B experiments)
LIB_PATH = os.environ.get("FTS_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libfts_gpu.so")

# fts_status (include/fts_gpu.h)
FTS_OK = 0
FTS_E_MALFORMED = 1
FTS_E_RP_NIL = 2
FTS_E_RP_INVALID = 3
FTS_E_IPA_NIL = 4
FTS_E_IPA_LEN = 5
FTS_E_IPA_INVALID = 6
FTS_E_RC_COUNT = 7
FTS_E_TAS_INVALID = 8
FTS_E_ST_INVALID = 9
FTS_E_NOT_RUN = 10
FTS_E_ACTION_INVALID = 11
FTS_E_OPEN_MISMATCH = 12
FTS_E_SIG_MALFORMED = 13
FTS_E_SIG_NOT_LOW_S = 14
FTS_E_SIG_INVALID = 15
FTS_E_NYM_MALFORMED = 16
FTS_E_NYM_BADKEY = 17
FTS_E_NYM_INVALID = 18
FTS_E_ID_MALFORMED = 19
FTS_E_ID_BADNYM = 20
FTS_E_ID_NO_EIDNYM = 21
FTS_E_ID_NO_RHNYM = 22
FTS_E_ID_REVOCATION = 23
FTS_E_ID_APRIME = 24
FTS_E_ID_PAIRING = 25
FTS_E_ID_ZK = 26
# mathlib CurveID of idemix issuer keys
FTS_CURVE_FP256BN_AMCL = 0
FTS_CURVE_BN254 = 1

FTS_API_OK = 0
FTS_DEVICE_NONE = -2
# prover seed: fresh getrandom() key per call (production); any other seed is test-only
FTS_SEED_OS_RANDOM = (1 << 64) - 1

EXPORTED = [
    "fts_ctx_create", "fts_ctx_create_bits", "fts_ctx_destroy", "fts_ctx_info",
    "fts_rp_verify_batch", "fts_transfer_verify_batch", "fts_issue_verify_batch", "fts_actions_verify_batch",
    "fts_rp_batch_stage", "fts_rp_batch_verify", "fts_rp_batch_free", "fts_rp_batch_merged", "fts_ctx_reserve", "fts_last_timings", "fts_last_timings_ex", "fts_rp_batch_timings",
    "fts_status_str", "fts_rp_prove", "fts_rp_prove_batch", "fts_token_commit",
    "fts_transfer_prove", "fts_issue_prove", "fts_debug_rp_intermediates",
    "fts_debug_msm_stats", "fts_msm_g1", "fts_msm_stage", "fts_msm_stage_multiples", "fts_msm_points", "fts_msm_run", "fts_msm_timings", "fts_msm_free",
    "fts_request_verify_batch", "fts_request_inspect", "fts_token_open_batch", "fts_rp_prove_batch_gpu",
    "fts_transfer_prove_batch_gpu", "fts_issue_prove_batch_gpu", "fts_token_metadata_open_batch",
    "fts_token_metadata_decode", "fts_ecdsa_verify_batch", "fts_ecdsa_sig_parse", "fts_p256_pubkey_from_pkix",
    "fts_ecdsa_last_timings", "fts_ctx_create_devices", "fts_ctx_create_mask", "fts_ctx_devices", "fts_shard_plan",
    "fts_idemix_ipk_create", "fts_idemix_ipk_destroy", "fts_nym_verify_batch", "fts_idemix_identity_nym",
    "fts_nym_last_timings", "fts_idemix_idv_create", "fts_idemix_idv_destroy", "fts_idemix_identity_verify_batch",
    "fts_idemix_identity_last_timings", "fts_idemix_identity_last_stats", "fts_idemix_pairing_debug", "fts_ctx_create_opts", "fts_debug_hold",
    "fts_debug_dispatch_stats", "fts_debug_stage_actions",
]


class PPInfo(C.Structure):
    _fields_ = [("bit_length", C.c_uint32), ("rounds", C.c_uint32), ("curve_id", C.c_uint32),
                ("device", C.c_int32), ("max_token", C.c_uint64), ("table_bytes", C.c_uint64),
                ("wide_bits", C.c_uint32), ("lanes", C.c_uint32)]


class CtxOpts(C.Structure):
    _fields_ = [("bit_length", C.c_uint32), ("wide_bits", C.c_int32), ("table_budget", C.c_uint64),
                ("lanes", C.c_int32), ("reserved", C.c_int32)]


class TransferItem(C.Structure):
    _fields_ = [("inputs", C.c_void_p), ("n_in", C.c_size_t), ("outputs", C.c_void_p), ("n_out", C.c_size_t),
                ("proof", C.c_void_p), ("proof_len", C.c_size_t)]


class IssueItem(C.Structure):
    _fields_ = [("tokens", C.c_void_p), ("n_tok", C.c_size_t), ("proof", C.c_void_p), ("proof_len", C.c_size_t)]


class TokenOpening(C.Structure):
    _fields_ = [("com64", C.c_void_p), ("type", C.c_void_p), ("type_len", C.c_size_t), ("value32", C.c_void_p),
                ("bf32", C.c_void_p)]


class EcdsaItem(C.Structure):
    _fields_ = [("msg", C.c_void_p), ("msg_len", C.c_size_t), ("sig", C.c_void_p), ("sig_len", C.c_size_t),
                ("pk64", C.c_void_p)]


class NymItem(C.Structure):
    _fields_ = [("nym", C.c_void_p), ("nym_len", C.c_size_t), ("sig", C.c_void_p), ("sig_len", C.c_size_t),
                ("msg", C.c_void_p), ("msg_len", C.c_size_t)]


class ActionWitness(C.Structure):
    _fields_ = [("type", C.c_void_p), ("type_len", C.c_size_t), ("n_in", C.c_size_t), ("in_values", C.c_void_p),
                ("in_bfs", C.c_void_p), ("n_out", C.c_size_t), ("out_values", C.c_void_p), ("out_bfs", C.c_void_p)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libfts_gpu.so not built: run `make -C fabric-token-sdk_amd` (%s)" % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    P, S, U8P, I32P = C.c_void_p, C.c_size_t, C.c_char_p, C.POINTER(C.c_int32)
    sig = {
        "fts_ctx_create": ([U8P, S, C.c_int, C.POINTER(P)], C.c_int),
        "fts_ctx_create_bits": ([U8P, S, C.c_uint32, C.c_int, C.POINTER(P)], C.c_int),
        "fts_ctx_destroy": ([P], None),
        "fts_ctx_info": ([P, C.POINTER(PPInfo)], C.c_int),
        "fts_ctx_create_opts": ([U8P, S, C.c_int, C.POINTER(CtxOpts), C.POINTER(P)], C.c_int),
        "fts_debug_hold": ([P, C.c_int], C.c_int),
        "fts_debug_dispatch_stats": ([P, C.POINTER(C.c_int64)], C.c_int),
        "fts_debug_stage_actions": ([P, S, C.POINTER(TransferItem), S, C.POINTER(IssueItem), C.c_int,
                                     C.POINTER(C.c_float)], C.c_int),
        "fts_rp_verify_batch": ([P, S, C.POINTER(C.c_void_p), C.POINTER(S), U8P, I32P], C.c_int),
        "fts_transfer_verify_batch": ([P, S, C.POINTER(TransferItem), I32P, I32P], C.c_int),
        "fts_issue_verify_batch": ([P, S, C.POINTER(IssueItem), I32P, I32P], C.c_int),
        "fts_actions_verify_batch": ([P, S, C.POINTER(TransferItem), S, C.POINTER(IssueItem), I32P, I32P, I32P, I32P],
                                     C.c_int),
        "fts_rp_batch_stage": ([P, S, C.POINTER(C.c_void_p), C.POINTER(S), U8P, C.POINTER(P)], C.c_int),
        "fts_rp_batch_verify": ([P, P, I32P], C.c_int),
        "fts_rp_batch_free": ([P], None),
        "fts_rp_batch_merged": ([P], C.c_int),
        "fts_ctx_reserve": ([P, S], C.c_int),
        "fts_last_timings": ([P, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.c_int], C.c_int),
        "fts_last_timings_ex": ([P, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.POINTER(C.c_double), C.c_int],
                                C.c_int),
        "fts_rp_batch_timings": ([P, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.POINTER(C.c_double), C.c_int],
                                 C.c_int),
        "fts_status_str": ([C.c_int32], C.c_char_p),
        "fts_rp_prove": ([P, C.c_uint64, U8P, C.c_uint64, P, S, C.POINTER(S), P], C.c_int),
        "fts_rp_prove_batch": ([P, S, C.POINTER(C.c_uint64), U8P, C.c_uint64, C.c_int, P, S, C.POINTER(S),
                                C.POINTER(S), P], C.c_int),
        "fts_token_commit": ([P, U8P, S, C.c_uint64, U8P, P], C.c_int),
        "fts_transfer_prove": ([P, U8P, S, S, C.POINTER(C.c_uint64), U8P, S, C.POINTER(C.c_uint64), U8P,
                                C.c_uint64, P, S, C.POINTER(S)], C.c_int),
        "fts_issue_prove": ([P, U8P, S, S, C.POINTER(C.c_uint64), U8P, C.c_uint64, P, S, C.POINTER(S)], C.c_int),
        "fts_debug_rp_intermediates": ([P, S, P, P, P], C.c_int),
        "fts_debug_msm_stats": ([P, C.POINTER(C.c_int64)], C.c_int),
        "fts_msm_g1": ([P, S, U8P, U8P, P], C.c_int),
        "fts_msm_stage": ([P, S, U8P, U8P, C.POINTER(P)], C.c_int),
        "fts_msm_stage_multiples": ([P, S, U8P, U8P, C.POINTER(P)], C.c_int),
        "fts_msm_points": ([P, P, S, S, P], C.c_int),
        "fts_msm_run": ([P, P, P], C.c_int),
        "fts_msm_timings": ([P, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.POINTER(C.c_double), C.c_int], C.c_int),
        "fts_msm_free": ([P], None),
        "fts_request_verify_batch": ([P, S, C.POINTER(C.c_void_p), C.POINTER(S), I32P, I32P, I32P], C.c_int),
        "fts_request_inspect": ([U8P, S, I32P, I32P, I32P, I32P, I32P, I32P], C.c_int),
        "fts_token_open_batch": ([P, S, C.POINTER(TokenOpening), I32P], C.c_int),
        "fts_token_metadata_open_batch": ([P, S, U8P, C.POINTER(C.c_void_p), C.POINTER(S), I32P], C.c_int),
        "fts_token_metadata_decode": ([U8P, S, I32P, C.POINTER(S), C.POINTER(S), P, P, I32P], C.c_int),
        "fts_transfer_prove_batch_gpu": ([P, S, C.POINTER(ActionWitness), C.c_uint64, P, S, C.POINTER(S),
                                          C.POINTER(S)], C.c_int),
        "fts_issue_prove_batch_gpu": ([P, S, C.POINTER(ActionWitness), C.c_uint64, P, S, C.POINTER(S),
                                       C.POINTER(S)], C.c_int),
        "fts_rp_prove_batch_gpu": ([P, S, C.POINTER(C.c_uint64), U8P, C.c_uint64, P, S, C.POINTER(S),
                                    C.POINTER(S), P], C.c_int),
        "fts_ecdsa_verify_batch": ([C.c_int, S, C.POINTER(EcdsaItem), I32P], C.c_int),
        "fts_ecdsa_sig_parse": ([U8P, S, P, P, I32P], C.c_int),
        "fts_p256_pubkey_from_pkix": ([U8P, S, P], C.c_int),
        "fts_ecdsa_last_timings": ([C.c_int, C.POINTER(C.c_float)], C.c_int),
        "fts_ctx_create_devices": ([U8P, S, C.c_uint32, I32P, C.c_int, C.POINTER(P)], C.c_int),
        "fts_ctx_create_mask": ([U8P, S, C.c_uint32, C.c_uint64, C.POINTER(P)], C.c_int),
        "fts_ctx_devices": ([P, I32P, C.c_int], C.c_int),
        "fts_shard_plan": ([S, C.POINTER(C.c_double), C.c_int, C.POINTER(S)], C.c_int),
        "fts_idemix_ipk_create": ([C.c_int, U8P, S, C.c_int, C.POINTER(P)], C.c_int),
        "fts_idemix_ipk_destroy": ([P], None),
        "fts_nym_verify_batch": ([P, S, C.POINTER(NymItem), I32P], C.c_int),
        "fts_idemix_identity_nym": ([U8P, S, C.POINTER(C.c_void_p), C.POINTER(S)], C.c_int),
        "fts_nym_last_timings": ([P, C.POINTER(C.c_float)], C.c_int),
        "fts_idemix_idv_create": ([C.c_int, U8P, S, C.c_int, C.POINTER(P)], C.c_int),
        "fts_idemix_idv_destroy": ([P], None),
        "fts_idemix_identity_verify_batch": ([P, S, C.POINTER(C.c_void_p), C.POINTER(S), I32P], C.c_int),
        "fts_idemix_identity_last_timings": ([P, C.POINTER(C.c_float)], C.c_int),
        "fts_idemix_identity_last_stats": ([P, C.POINTER(C.c_uint32)], C.c_int),
        "fts_idemix_pairing_debug": ([P, C.c_int, U8P, C.c_int, C.POINTER(C.c_uint32)], C.c_int),
    }
    for name, (args, res) in sig.items():
        try:
            f = getattr(lib, name)
        except AttributeError:
            if os.environ.get("FTS_LIB"):  # an A/B build of an older revision: its missing entries stay unbound
                continue
            raise
        f.argtypes = args
        f.restype = res
    return lib


lib = _load()


class FtsError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__("%s failed with API code %d" % (fn, code))
        self.code = code


def check(fn, code):
    if code != FTS_API_OK:
        raise FtsError(fn, code)


def shard_plan(n, nshards, weights=None):
    """fts_shard_plan: contiguous shard bounds [b_0 = 0, ..., b_nshards = n]"""
    b = (C.c_size_t * (nshards + 1))()
    w = (C.c_double * n)(*weights) if weights is not None else None
    check("fts_shard_plan", lib.fts_shard_plan(n, w, nshards, b))
    return list(b)


def status_str(s):
    return lib.fts_status_str(int(s)).decode()
