#!/bin/bash
# round 4: the whole -m gpu suite (as the driver runs it, verbose) and smoke()
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -rP > $O/tests.txt 2>&1
echo suite done
timeout -k 10 90 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo smoke done
