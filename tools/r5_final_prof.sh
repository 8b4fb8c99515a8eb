# Round-5 final: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE PMC passes of the default bench command (cifar10) and
# of the POWER bench, on the final kernel sources (tools/profile_round.sh)
set -e
R=$GRAFT_REPO_ROOT
bash $R/tools/profile_round.sh r05fc
bash $R/tools/profile_round.sh r05fp --config power
