"""bench.py's output contract on CPU: rank 0 prints exactly one JSON line on stdout, so C-level prints made
while the RCCL communicator is created (its version banner) must land on stderr."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stdout_to_stderr_covers_c_level_writes():
    code = (
        "import os, sys\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "q = bench._StdoutToStderr()\n"
        "q.__enter__()\n"
        "os.write(1, b'RCCL version : banner\\n')\n"
        "print('python-level noise')\n"
        "q.__exit__()\n"
        "print('{\"metric\": \"m\"}')\n" % ROOT
    )
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"metric": "m"}']
    assert "RCCL version" in r.stderr and "python-level noise" in r.stderr
