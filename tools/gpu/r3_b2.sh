#!/bin/bash
# flat column groups A/B + GW merge restructure
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu/r3_flatw.sh || exit 1
bash tools/gpu/r3_gwm.sh
