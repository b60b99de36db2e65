bash tools/sweep.sh 1e9
