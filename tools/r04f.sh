#!/bin/bash
# round-4 batch f (GPU box): stream-priority A/B of the bench step, host-side cProfile of the step
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04f
timeout -k 10 400 python -u tools/priority_ab.py 8 > gpurun_out/${t}_priority_ab.log 2>&1 || { rc=$?; tail -20 gpurun_out/${t}_priority_ab.log; exit $rc; }
tail -6 gpurun_out/${t}_priority_ab.log
timeout -k 10 300 python -u tools/host_profile.py 5 > gpurun_out/${t}_host_profile.log 2>&1 || exit $?
head -3 gpurun_out/${t}_host_profile.log
