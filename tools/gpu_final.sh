#!/bin/bash
# Round evidence for HEAD (see tools/gpu_run.sh for the steps).
bash "${GRAFT_REPO_ROOT:-.}/tools/gpu_run.sh" ${TAG:-final} pytest bench bench4 fp32 rankshare traffic valu prof
exit $?
