#!/bin/sh
# move2kube_amd detector: Node.js project (package.json).
test -f "$1/package.json" || exit 1
printf '%s\n' '{"port": 8080, "app_name": "app"}'
