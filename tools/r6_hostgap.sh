#!/bin/bash
# host time of a CIFAR-10 eval step's start (tools/r6_hostgap.py) on the GPU box
set -o pipefail
mkdir -p gpurun_out/r6_hostgap
timeout -k 10 300 python -u tools/r6_hostgap.py 20 > gpurun_out/r6_hostgap/${1:-base}.txt 2>&1
