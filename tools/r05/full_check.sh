#!/bin/bash
# The round-end checks the driver runs, ahead of it: the whole GPU suite,
# smoke(), and the default bench line.  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
tail -c 600 $O/bench.json
echo "full check done"
