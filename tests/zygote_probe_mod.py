"""Container module for tests/test_zygote.py: reports what the forked process sees."""
import json
import os
import sys

import numpy
import torch
from threadpoolctl import threadpool_info

numpy.ones((256, 256)) @ numpy.ones((256, 256))  # the BLAS pool works after the fork
blas = [d["num_threads"] for d in threadpool_info() if d["user_api"] == "blas"]

print("PROBE " + json.dumps({"threads": torch.get_num_threads(), "blas_threads": blas[:1],
                             "cpus": sorted(os.sched_getaffinity(0)),
                             "env": os.environ.get("PROBE_VAR"), "argv": sys.argv[1:], "cwd": os.getcwd()}), flush=True)
sys.exit(int(os.environ.get("PROBE_EXIT", "0")))
