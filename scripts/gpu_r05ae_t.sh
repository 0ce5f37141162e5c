#!/bin/bash
# round 5: fp32 rows on the wide chain and the row-format bit-equality test, then the whole -m gpu suite
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05ae_t}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_hip_parity.py -k "row_formats or fp32_rows" -x -v --timeout 120 --timeout-method thread > $O/pytest_rowfmt.log 2>&1 || { tail -40 $O/pytest_rowfmt.log; exit 1; }
tail -1 $O/pytest_rowfmt.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
