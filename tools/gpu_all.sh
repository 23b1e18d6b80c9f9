#!/bin/bash
# evidence pass + N=2 rehearsal in one call
cd "$GRAFT_REPO_ROOT" || exit 3
./tools/gpu_round_profile.sh || exit $?
./tools/gpu_rehearse_n2.sh || exit $?
