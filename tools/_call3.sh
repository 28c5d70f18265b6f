# r05 session: products k = 64 / 32 backward depth A/B: base (depth from the average degree:
# phase 1 U = 8, phase 2 U = 8 at k = 64), x4 (phase 1 U = 4), su4 (phase 2 U = 4), xs4 (both),
# x16 (phase 1 U = 16)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s22
mkdir -p $O
R=2 timeout -k 10 1100 bash tools/ab_bench.sh "base x4 su4 xs4 x16" "--graph products --k 64" "--graph products --k 32" > $O/ab.txt 2>&1
cat $O/ab.txt
