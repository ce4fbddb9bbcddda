#!/bin/sh
# move2kube_amd detector: PHP sources anywhere below the directory.
src="$1"
n=$(find "$src"/. -name '*.php' -print 2>/dev/null | head -n 1 | wc -l)
[ "$n" -eq 1 ] || exit 1
printf '%s\n' '{"port": 8080, "binding": "0.0.0.0:8080", "app_name": "app"}'
