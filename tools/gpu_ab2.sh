#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/ab_kstats.sh ${1:-2}
