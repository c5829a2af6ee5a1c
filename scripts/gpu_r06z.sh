#!/bin/bash
# Round 6: the GPU suite and smoke() on the final tree (the round-end check, run ahead of the driver).
set -o pipefail
mkdir -p gpurun_out/r06z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06z/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06z/smoke.log 2>&1
