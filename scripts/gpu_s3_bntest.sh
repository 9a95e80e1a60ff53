#!/bin/bash
set -u
timeout -k 10 300 python -u -m pytest tests/test_batchnorm_gpu.py -x -q --timeout 120 --timeout-method thread
