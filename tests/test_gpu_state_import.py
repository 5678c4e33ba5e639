"""Exploit import from a side stream into a captured step: tools/import_check.py in the
deterministic build (two members with the same state / batch / hyperparameters then step bitwise identically), in a
subprocess because the kernel library is chosen when it is first loaded.

ProcessGroupNCCL receives into the destination state row on its own communication stream and ``work.wait()`` orders
the current stream after it; parallel/dataplane.py relies on that plus ``PopulationEngine.on_state_imported`` (host
step counter, bf16 weight-shadow refresh) before the next REPLAY of the captured step graph.  The check issues the
copy on a side stream that is still busy when the replay is enqueued, and requires the importing member to come out
of the replayed step bitwise equal to the source member, at the source's step counter.  Reference behaviour:
/root/reference/pbt_cluster.py:145-164 (the exploited member continues from the winner's checkpoint and step).
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_side_stream_import_then_graph_replay():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DTF_DETERMINISTIC="1", DTF_HIP_GRAPH="1")
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "import_check.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    print(r.stdout[-2000:])
    assert r.returncode == 0 and "IMPORT_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
