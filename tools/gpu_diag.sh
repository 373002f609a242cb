#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u "$@" > gpurun_out/diag.log 2>&1; rc=$?; tail -40 gpurun_out/diag.log; exit $rc
