#!/bin/bash
# HAR encoder after the round-5 swizzle: rocprofv3 kernel stats, then the four PMC passes.
set -o pipefail
bash tools/rocprof_har.sh && echo "rocprof ok" && bash tools/pmc_har.sh && echo "pmc ok"
