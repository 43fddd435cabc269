#!/bin/bash
# Stand-in for ssh in the launcher's --cluster ssh test: drops ssh options, takes the host and
# runs the remote command locally in a clean environment (as a remote login shell would have),
# exposing the host name it was "sent" to as FAKE_SSH_HOST.
while [ $# -gt 0 ]; do
  case $1 in
    -o) shift 2 ;;
    -*) shift ;;
    *) break ;;
  esac
done
host=$1; shift
exec env -i PATH="$PATH" HOME="$HOME" FAKE_SSH_HOST="$host" \
  HIP_VISIBLE_DEVICES="" CUDA_VISIBLE_DEVICES="" bash -c "$*"
