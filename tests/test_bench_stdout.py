"""bench.py's stdout contract: the driver reads ONE JSON line.  Native libraries (RCCL's version banner at
communicator init) write to file descriptor 1; bench.quiet_native_stdout() points fd 1 at stderr and
bench.emit() writes the line to a duplicate of the original stdout."""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_one_json_line_despite_native_stdout_writes():
    code = (
        "import os, sys\n"
        f"sys.path.insert(0, {str(ROOT)!r})\n"
        "import bench\n"
        "bench.quiet_native_stdout()\n"
        "os.write(1, b'RCCL version : banner on fd 1\\n')\n"
        "print('python print after the redirect')\n"
        "bench.emit({'metric': 'm', 'value': 1.0})\n"
    )
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    assert json.loads(lines[0]) == {"metric": "m", "value": 1.0}
    assert "RCCL version" in r.stderr and "python print" in r.stderr
