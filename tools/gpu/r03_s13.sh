#!/bin/bash
# r03 session 13: validation of the final tree (GPU tests, smoke, bench), then
# clock/power under the headline step
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/validate.sh || exit $?
bash tools/gpu/power_sample.sh
