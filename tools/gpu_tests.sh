#!/bin/bash
# GPU test run for gpurun: the drop-in test first, then the whole -m gpu suite.
# pytest exit 0 (pass) or 1 (failures) lets the next step run; anything else
# (a timeout, a crash, an interrupted run) ends the script there.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py -v --timeout 300 --timeout-method thread \
    > gpurun_out/gt_dropin.log 2>&1
rc=$?
echo "dropin rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    --deselect tests/test_gpu_dropin.py > gpurun_out/gt_all.log 2>&1
rc2=$?
echo "all rc=$rc2"
tail -5 gpurun_out/gt_all.log
exit $(( rc > rc2 ? rc : rc2 ))
