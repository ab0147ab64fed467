#!/bin/bash
# Reference compat (scripts/stop.sh kill -9s every xflow_lr): stop only the
# worker processes this user started from this checkout, by PID file if the
# launcher wrote one, never by command-line pattern.
pidfile=${XFLOW_PIDFILE:-/tmp/xflow_workers.pid}
[ -f "$pidfile" ] || { echo "no pid file $pidfile"; exit 0; }
while read -r p; do kill "$p" 2>/dev/null; done < "$pidfile"
rm -f "$pidfile"
