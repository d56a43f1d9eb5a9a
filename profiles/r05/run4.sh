#!/bin/bash
set -eo pipefail
bash profiles/r05/shares.sh r05 c3 8 0 1 2 3 4 5 6 7
