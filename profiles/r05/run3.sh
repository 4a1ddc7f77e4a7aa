#!/bin/bash
# round 5, call 3: block-stagger A/B (the knob is now read in every build)
cd "$(dirname "$0")/../.."
bash profiles/r05/env_ab.sh stag3 "" "HFG_STAGGER=25,0" "HFG_STAGGER=50,0" "HFG_STAGGER=0,10" "HFG_STAGGER=0,25" "HFG_STAGGER=40,15"
