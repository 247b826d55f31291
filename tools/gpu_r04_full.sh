#!/bin/bash
# round 4: the whole -m gpu suite + smoke() (as the driver runs them), then the default bench line with its
# rocprofv3 kernel trace and PMC traffic passes
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r04f}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -rP > $O/tests.txt 2>&1
echo suite done
timeout -k 10 90 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo smoke done
bash tools/gpu.sh c2 ${1:-r04f}
echo c2 done
