"""CPU ORACLE — test infrastructure only.

This package is a from-scratch CPU restatement of the reference verification
path of the zkatdlog "nogh" driver (fabric-token-sdk @ 2025-03-21) and of the
BN254 arithmetic it delegates to IBM/mathlib -> gnark-crypto v0.13.0.

It is used ONLY by ``tests/``, by ``__graft_entry__.smoke()`` and by the
``cpu_baseline`` leg of ``bench.py`` — as the checker, never as the thing that
is measured or shipped.  The product path (``fabric-token-sdk_amd/``) never
imports it and fails loudly when its HIP library is missing.

Pinning: ``oracle.bn254.hash_to_g1`` reproduces all 130 range-proof generators
of the reference fixture ``cmd/tokengen/testdata/zkatdlog_pp.json`` (KAT-1,
``tests/test_oracle.py``).  Everything above the curve arithmetic
(HashToZr, Zr byte encoding, transcripts) has no golden vector in the
reference and is "parity unpinned" beyond the KAT — see DESIGN.md §Oracle.
"""
