# A/B of the tree's library against alternative builds gpurun_alt/lib_<name>.so: paired-series time per term and
# phase stamps at CIFAR scales 0 and 1 (B=64), then the 128-pixel parity subset on the tree's library.
#   bash tools/exp_ab.sh <name> ...
cd $GRAFT_REPO_ROOT
bash tools/exp_attr_k128.sh "$@" || exit 1
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py -k "k128 or headline or golden or overlap" 2>&1 | tail -5
