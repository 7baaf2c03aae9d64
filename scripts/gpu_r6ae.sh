#!/bin/bash
# Round 6: the GPU test suite on the device-check build (QFEDX_DEBUG=1: _qfedx_C_debug, QFX_DCHECK bounds checks that
# raise after a failing launch).
source "$(dirname "$0")/gpu_step.sh"
QFEDX_DEBUG=1 TAILN=3 step dbg_tests 1000 env QFEDX_DEBUG=1 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
