#!/bin/bash
# Reference compat (scripts/start_server.sh): servers have no work here --
# every worker rank serves a shard of the HBM table.  Kept so existing
# cluster recipes run unchanged.  usage: start_server.sh <num_servers> <bin> [args..]
n=${1:-1}; shift
for ((i=0; i<n; ++i)); do DMLC_ROLE=server "$@" & done
wait
