"""The in-process N-device path (one JVM driving every GPU of a
node through one context, cordahip_init(0xFF...)) executed on a one-GPU box:
cordahip_init's test knob CORDAHIP_TEST_DEVICE_REPLICAS=k gives the context k
Device objects on HIP device 0, each with its own streams, workspaces and
tables, so the shard split, one worker per device, ragged shard tails and the
reassembly of statuses / verdict words run for real. tests/multidev_worker.py
drives the generic CSR batch (both sections), the dense host rows, tx ids,
signed transactions (leaves and components: each device's own encoder state,
the templates-only chain from the third call), filtered transactions and the
C5 stream, and compares every result
with the goldens / oracle and with a one-device context. Small pipeline chunks
(CORDAHIP_HOST_CHUNK / CORDAHIP_STREAM_CHUNK) make every shard span several
chunks and reuse all pipeline stages; CORDAHIP_TX_SLICES=5 runs every device's
tx ids of a signed-tx batch as 5 asynchronous slices feeding the signatures."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("replicas", [2, 3])
def test_multi_device_context(replicas):
    env = dict(os.environ, CORDAHIP_TEST_DEVICE_REPLICAS=str(replicas), CORDAHIP_HOST_CHUNK="256",
               CORDAHIP_STREAM_CHUNK="512", CORDAHIP_TX_SLICES="5",
               CORDAHIP_TX_SIG_CHUNK="5")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "multidev_worker.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["device_count"] == replicas and not out["bad"]
