#!/bin/bash
# Count MFMA vs 32x32->64 MAD instructions in the gfx950 code objects (no GPU needed).
set -e
cd "$(dirname "$0")/../fabric-token-sdk_amd"
for f in rp_kernels msm sigma_kernels; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only --no-gpu-bundle-output \
    -x hip -c csrc/$f.hip -o /tmp/isa_$f.o
  dis=$(/opt/rocm/lib/llvm/bin/llvm-objdump -d /tmp/isa_$f.o)
  echo "$f: v_mfma=$(grep -c v_mfma <<< "$dis" || true) v_mad_u64_u32=$(grep -c v_mad_u64_u32 <<< "$dis" || true)"
done
