"""Runtime settings the package applies at import (dbx_distributed_pytorch_examples_amd/__init__.py):
two HIP graph queues unless the environment already names a count (profiles/r4_final2/README.md)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_PROBE = "import os, dbx_distributed_pytorch_examples_amd; print(os.environ.get('DEBUG_HIP_FORCE_GRAPH_QUEUES'))"


def _probe(env_extra):
    env = {k: v for k, v in os.environ.items() if k != "DEBUG_HIP_FORCE_GRAPH_QUEUES"}
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", _PROBE], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


def test_graph_queue_default_set_at_import():
    assert _probe({}) == "2"


def test_graph_queue_explicit_setting_wins():
    assert _probe({"DEBUG_HIP_FORCE_GRAPH_QUEUES": "1"}) == "1"
