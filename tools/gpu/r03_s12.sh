#!/bin/bash
# r03 session 12: profile round on the split-iteration tree, then clock/power
# under the headline step
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/profile_round.sh || exit $?
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/power_sample.sh
