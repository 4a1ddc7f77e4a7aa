#!/bin/bash
# round 5, call 1: GPU suite + smoke, then the block-stagger A/B
cd "$(dirname "$0")/../.."
bash profiles/r05/suite.sh || exit $?
bash profiles/r05/env_ab.sh stag "" "HFG_STAGGER=5,0" "HFG_STAGGER=10,0" "HFG_STAGGER=0,3" "HFG_STAGGER=0,8"
