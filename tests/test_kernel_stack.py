"""Guard: no kernel of libcordahip.so may use a dynamic stack.

The first GPU build of the Kryo encoder flushed its nested OutputChunked levels
recursively; the compiler gave the kernel a dynamic stack, which overflowed and
faulted the GPU. kryo_core.hpp now bounds the cascade with a static-depth
template chain. This reads the kernel descriptors of every gfx950 code object
in the built library (tools/kernel_notes.py: `.uses_dynamic_stack`,
`.private_segment_fixed_size` from the AMDGPU metadata note) and fails if a
dynamic stack appears anywhere, or if the encoder kernels' fixed private
segments grow past a bound (a recursion the compiler could not size would show
up as a dynamic stack; a runaway static one as a large fixed size).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "corda_amd", "libcordahip.so")

# bytes of fixed private segment a kernel may use (the Kryo kernels' level
# bookkeeping and graph tables; scratch is memory traffic, so keep it small)
MAX_PRIVATE = 4096


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.skip("libcordahip.so not built")
    import kernel_notes

    ks = kernel_notes.library_kernels(LIB)
    assert ks, "no gfx950 kernels found in libcordahip.so"
    return ks


def test_no_dynamic_stack(kernels):
    bad = [k["name"] for k in kernels if k[".uses_dynamic_stack"]]
    assert not bad, "kernels with a dynamic stack: %s" % bad


def test_private_segments_bounded(kernels):
    big = [(k["name"], k[".private_segment_fixed_size"]) for k in kernels
           if k[".private_segment_fixed_size"] > MAX_PRIVATE]
    assert not big, big


def test_product_kernels_present(kernels):
    names = " ".join(k["name"] for k in kernels)
    for kern in ("ed25519_prep_half_kernel", "ed25519_ladder_half_kernel", "ecdsa_ladder_kernel",
                 "sha256_leaves_kernel", "merkle_root_kernel", "kryo_"):
        assert kern in names, kern
