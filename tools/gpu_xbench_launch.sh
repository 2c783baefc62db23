#!/bin/bash
# round 5: host cost of one kernel launch by API, and through the engine library with / without torch
set -o pipefail
timeout -k 10 120 tools/launchbench/launch_bench | head -4 && timeout -k 10 200 python3 -u tools/xbench_launch.py
