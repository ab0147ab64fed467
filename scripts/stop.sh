#!/bin/bash
# Reference compat (scripts/stop.sh kill -9s every xflow_lr): stop exactly the
# processes scripts/local.sh started (it records their PIDs in the pid file),
# never by command-line pattern.  SIGTERM first, SIGKILL after a grace period.
pidfile=${XFLOW_PIDFILE:-/tmp/xflow_workers.$(id -u).pid}
[ -f "$pidfile" ] || { echo "no pid file $pidfile"; exit 0; }
mapfile -t pids < "$pidfile"
for p in "${pids[@]}"; do kill "$p" 2>/dev/null; done
for _ in 1 2 3 4 5 6 7 8 9 10; do
    alive=0
    for p in "${pids[@]}"; do kill -0 "$p" 2>/dev/null && alive=1; done
    [ $alive = 0 ] && break
    sleep 0.5
done
for p in "${pids[@]}"; do kill -9 "$p" 2>/dev/null; done
rm -f "$pidfile"
echo "stopped ${#pids[@]} process(es)"
