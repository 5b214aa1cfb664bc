#!/bin/bash
# round 4: k_schur item size A/B (MCC_ITEM_SLOTS) on configs 4, 5, 3 with one hand-off level
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/ab_trees.sh config4 2 HEAD "HEAD:MCC_ITEM_SLOTS=128" "HEAD:MCC_ITEM_SLOTS=64" "HEAD:MCC_ITEM_SLOTS=32" || exit 12
bash tools/ab_trees.sh config5 2 HEAD "HEAD:MCC_ITEM_SLOTS=128" "HEAD:MCC_ITEM_SLOTS=64" || exit 13
