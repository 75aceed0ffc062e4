#!/bin/bash
# Build A/B variants of libcordahip.so into ab_libs/<tag>/libcordahip.so (CPU,
# in this container; the .so files travel to the GPU box, tools/gpu_ab.sh swaps
# them in). Usage: tools/build_ab.sh <tag> "<extra flags for every TU>" "<extra ladder flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
tag=$1
mkdir -p "$R/ab_libs/$tag" "$R/build/ab/$tag"
# the variants differ only in the translation units named in $REBUILD (default:
# the Ed25519 ones): reuse the main build's other objects (make sees them newer
# than their sources)
REBUILD=${REBUILD:-"ed25519 ed25519_ladder"}
for o in ed25519 ed25519_ladder ecdsa tx cordahip kryo; do [ -f "$R/build/obj/$o.o" ] && cp -p "$R/build/obj/$o.o" "$R/build/ab/$tag/"; done
for o in $REBUILD; do rm -f "$R/build/ab/$tag/$o.o"; done
make -s -j8 -C "$R/corda_amd/csrc" OUT="$R/ab_libs/$tag/libcordahip.so" OBJDIR="$R/build/ab/$tag" \
  EXTRA_FLAGS="$2" LADDER_FLAGS="$3" 2>&1 | grep -v "loop not unrolled\|warnings generated" || true
ls -la "$R/ab_libs/$tag/libcordahip.so"
