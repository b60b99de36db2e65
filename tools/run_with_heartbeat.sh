#!/bin/bash
# Runs a long GPU command that prints rarely (the C++ drop-in matrix at
# maxNum 1e6) with a heartbeat line every 50 s in <dir>/heartbeat.txt, so that
# gpurun's silence watchdog does not take it for hung; the command keeps its
# own time limit and writes its output to <dir>/<name>.txt.
# usage: tools/run_with_heartbeat.sh <dir> <name> <seconds> cmd...
DIR=$1; NAME=$2; LIM=$3; shift 3
mkdir -p "$DIR"
(while sleep 50; do date >> "$DIR/heartbeat.txt"; done) &
HB=$!
timeout -k 10 "$LIM" "$@" > "$DIR/$NAME.txt" 2>&1
rc=$?
kill $HB
echo "$NAME rc=$rc"
tail -4 "$DIR/$NAME.txt"
exit $rc
