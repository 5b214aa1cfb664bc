set -o pipefail
tools/env_ab.sh config4 2 "MCC_GROUP_EDGES=16" "MCC_GROUP_EDGES=8" "MCC_GROUP_EDGES=4" "MCC_GROUP=0" || exit 1
tools/env_ab.sh config5 2 "MCC_GROUP=1" "MCC_GROUP=1 MCC_GROUP_EDGES=8" "MCC_GROUP=0" || exit 1
tools/env_ab.sh config3 1 "MCC_GROUP=1" "MCC_GROUP=0" || exit 1
