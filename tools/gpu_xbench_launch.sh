#!/bin/bash
# Host cost of one kernel launch by HIP API (tools/launchbench) and through the engine library with torch loaded
set -o pipefail
timeout -k 10 120 tools/launchbench/launch_bench | head -4 && timeout -k 10 200 python3 -u tools/xbench_launch.py
