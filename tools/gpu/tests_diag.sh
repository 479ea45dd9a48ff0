#!/bin/bash
# GPU box: the given test files (-m gpu), then, if green, tools/gpu/diag.sh on
# the given configs. Usage: tests_diag.sh "<pytest files>" <config>...
set -o pipefail
TESTS=$1; shift
bash tools/gpu/suite.sh $TESTS || exit $?
[ $# -gt 0 ] && bash tools/gpu/diag.sh "$@"
