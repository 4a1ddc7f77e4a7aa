#!/bin/bash
cd "$(dirname "$0")/../.."
bash profiles/r04/run12.sh && bash profiles/r04/run8.sh
