#!/bin/bash
# Run a command with environment assignments (lease.sh sh: steps take no env):
#   bash tools/env_run.sh VAR=value ... <command> [args]
exec env "$@"
