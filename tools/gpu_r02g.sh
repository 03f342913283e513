bash tools/pmc_round.sh r02g || exit 1
