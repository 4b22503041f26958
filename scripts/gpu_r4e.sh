#!/bin/bash
# r4b (exchange engines) then r4d (BERT / async PS) in one call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r4e} bash scripts/gpu_r4b.sh && TAG=${TAG:-r4e} bash scripts/gpu_r4d.sh
