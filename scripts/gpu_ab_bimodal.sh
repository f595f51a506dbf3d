#!/bin/bash
# In-process A/B of persistent-kernel build variants on the bimodal batch
set -u
O=gpurun_out/abb; mkdir -p $O
AB_WORKLOAD=bimodal timeout -k 10 400 python -u scripts/ab_inproc.py hysteria_amd/libhyobfs.so:persistent "$@" > $O/ab.txt 2>&1
echo rc=$?
