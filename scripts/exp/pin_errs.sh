#!/bin/bash
# the default headline update's fp32 pin, with its per-parameter relative update errors printed
timeout -k 10 300 python -u -m pytest -s -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_learning.py::test_default_headline_update_matches_fp32_torch_update" 2>&1 | grep -E "relative|native stats|passed|failed"
