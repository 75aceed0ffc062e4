#!/bin/bash
# Build A/B variants of libcordahip.so into ab_libs/<tag>/libcordahip.so (CPU,
# in this container; the .so files travel to the GPU box, tools/gpu_ab.sh swaps
# them in). Usage: tools/build_ab.sh <tag> "<extra flags for every TU>" "<extra ladder flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
tag=$1
mkdir -p "$R/ab_libs/$tag" "$R/build/ab/$tag"
# the variants differ only in the Ed25519 translation units: reuse the main
# build's other objects (make sees them newer than their sources)
for o in ecdsa tx cordahip; do [ -f "$R/build/obj/$o.o" ] && cp -p "$R/build/obj/$o.o" "$R/build/ab/$tag/"; done
rm -f "$R/build/ab/$tag/ed25519.o" "$R/build/ab/$tag/ed25519_ladder.o"
make -s -j8 -C "$R/corda_amd/csrc" OUT="$R/ab_libs/$tag/libcordahip.so" OBJDIR="$R/build/ab/$tag" \
  EXTRA_FLAGS="$2" LADDER_FLAGS="$3" 2>&1 | grep -v "loop not unrolled\|warnings generated" || true
ls -la "$R/ab_libs/$tag/libcordahip.so"
