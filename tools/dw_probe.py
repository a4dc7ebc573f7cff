"""The weight-gradient group of one go2 minibatch alone (bench.py learner_gemm_roofline), for
rocprofv3 kernel-trace / PMC passes (dev tool): python tools/dw_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(bench.learner_gemm_roofline("cuda:0"))
