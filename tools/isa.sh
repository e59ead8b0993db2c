#!/bin/bash
# Device ISA of the product kernels with the Makefile's flags: tools/isa.sh OUT.s [extra hipcc flags]
cd "$(dirname "$0")/../surf-path-tracer_amd" || exit 1
OUT=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -I../include -Icsrc "$@" \
  -S --cuda-device-only csrc/surf_hip.hip -o "$OUT"
