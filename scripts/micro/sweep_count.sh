export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 16 32; do for w in 0 1; do HD_JACOBI_WARM=$w timeout -k 10 120 python scripts/micro/sweep_count.py $n; done; done
