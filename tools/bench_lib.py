#!/usr/bin/env python3
"""Run bench.py against a design-experiment library (tools only): bench_lib.py LIB [bench args].
The product loader reads no environment variable; this binds LIB through _lib.use_library()
before bench.py imports the package."""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from audiorenderingv2_amd._lib import use_library  # noqa: E402

use_library(sys.argv[1])
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
