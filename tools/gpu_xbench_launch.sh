#!/bin/bash
# Host cost of one kernel launch by HIP API (tools/launchbench) and through the engine library with torch loaded
# (build first: hipcc -O2 --offload-arch=gfx950 tools/launchbench/launch_bench.hip -o tools/launchbench/launch_bench)
set -o pipefail
timeout -k 10 120 tools/launchbench/launch_bench && timeout -k 10 200 python3 -u tools/xbench_launch.py
