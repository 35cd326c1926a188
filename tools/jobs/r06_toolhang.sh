#!/bin/bash
set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "policy_variants" 2>&1 | tail -15
