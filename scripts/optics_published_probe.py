#!/usr/bin/env python3
"""OPTICS on the published benchmark workloads (bench.bench_optics_published) alone."""
import sys, json
sys.path.insert(0, "event-camera-clustering-and-optical-flow-estimation_amd"); sys.path.insert(0, ".")
import eccpy as ecc
import bench
ctx = ecc.Context(0)
print(json.dumps(bench.bench_optics_published(ecc, ctx), indent=1))
