#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ref_opencl.py -m gpu -q -rf > gpurun_out/pytest_ref.log 2>&1; rc=$?; echo "pytest_ref rc=$rc"; tail -4 gpurun_out/pytest_ref.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash scripts/gpu_profile.sh r01
