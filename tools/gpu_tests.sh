#!/bin/bash
# the whole GPU suite with the test prints kept (-s), failures listed
set -o pipefail
O=gpurun_out
tag="${1:-r04}"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_$tag.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 $O/tests_$tag.log; grep -E "^FAILED" $O/tests_$tag.log
exit $rc
