#!/bin/bash
# Stand-in for mpirun in the launcher's --cluster mpi test: `-n N cmd...` starts N copies of the
# command with Open MPI's rank variables (two "nodes" of N/2 ranks each) and waits for them all.
n=1
while [ $# -gt 0 ]; do
  case $1 in
    -n|-np) n=$2; shift 2 ;;
    -*) shift ;;
    *) break ;;
  esac
done
half=$(( (n + 1) / 2 ))
pids=()
for ((r = 0; r < n; r++)); do
  OMPI_COMM_WORLD_RANK=$r OMPI_COMM_WORLD_SIZE=$n OMPI_COMM_WORLD_LOCAL_RANK=$(( r % half )) \
    OMPI_COMM_WORLD_LOCAL_SIZE=$half "$@" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
exit $rc
