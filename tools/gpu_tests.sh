#!/bin/bash
# Run GPU test files one after another; stop at the first crash (not at test failures).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for f in "$@"; do
  timeout -k 10 600 python -m pytest "$f" -q -m gpu -rf --maxfail=40 -p no:cacheprovider > "gpurun_out/$(basename $f .py).log" 2>&1
  rc=$?
  tail -30 "gpurun_out/$(basename $f .py).log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $f exited $rc"; exit $rc; fi
done
exit 0
