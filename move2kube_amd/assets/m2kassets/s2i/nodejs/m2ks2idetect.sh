#!/bin/sh
# move2kube_amd S2I detector: Node.js (package.json).
test -f "$1/package.json" || exit 1
printf '{"builder": "%s", "port": 8080}\n' "registry.access.redhat.com/ubi8/nodejs-10"
