#!/bin/bash
# usage: scripts/asm.sh SRC.hip OUT.s [extra hipcc flags]: gfx950 device ISA listing
D=/root/repo/ece1782-smith-waterman-cuda_amd/csrc
src=$1; out=$2; shift 2
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fvisibility=hidden -DSW_AMD_BUILD -I/root/repo/include -I$D --cuda-device-only -S -o "$out" "$D/$src" "$@" 2>&1 | grep -E "error" -A3
true
