#!/bin/sh
# move2kube_amd detector: Django application (Pipfile based).
# Protocol: $1 = candidate source directory; exit 0 + JSON on stdout = match.
src="$1"
test -f "$src/Pipfile" || exit 1
printf '%s\n' '{"port": 8080, "binding": "0.0.0.0:8080"}'
