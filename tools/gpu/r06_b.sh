#!/bin/bash
# Round 6, VERDICT r05 W6: does the exit-time SIGSEGV under rocprofv3 follow a cooperative
# launch without any n2v2r code?  tools/coop_exit_repro (built on the CPU host): one trivial
# kernel launched plainly, then cooperatively, each under rocprofv3's kernel trace.  The plain
# run goes first; the cooperative one (the one expected to crash at exit) last, and nothing runs
# on the GPU after it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_b
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/plain -o run -- ./tools/coop_exit_repro plain > $O/plain.log 2>&1
echo "plain rc=$?" | tee -a $O/rc.txt
[ "$(tail -1 $O/rc.txt)" = "plain rc=0" ] || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/coop -o run -- ./tools/coop_exit_repro coop > $O/coop.log 2>&1
echo "coop rc=$?" | tee -a $O/rc.txt
exit 0
