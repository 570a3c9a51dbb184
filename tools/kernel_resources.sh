#!/bin/bash
# SGPR/VGPR/scratch use of every gfx950 kernel in jsp_kernels.hip (device-only compile, no GPU needed)
set -e
out=$(mktemp /tmp/jspk.XXXXXX.co)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -c \
    -o "$out" "$(dirname "$0")/../jobset_amd/csrc/${KFILE:-jsp_kernels.hip}" 2>/dev/null
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$out" |
    grep -E "^\s+\.name:|private_segment_fixed_size|\.sgpr_count|\.vgpr_count" | paste - - - - |
    sed -E 's/ +/ /g; s/\.name: _ZN3jsp[0-9]+//' | grep -E "${1:-.}"
rm -f "$out"
