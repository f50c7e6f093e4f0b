#!/bin/bash
# --pmc progress: simulations in chunks (no selfplay step) vs one selfplay step, 256 games x 800 sims
set -o pipefail
cd "$(dirname "$0")/.."
TAG=probe4 CFGS="256:800:800:sims:0 256:800:0:step:0" timeout -k 10 400 tools/pmc_hang_probe2.sh 2>&1 | grep -v "^  File\|^Thread\|^Timeout" | tail -12
