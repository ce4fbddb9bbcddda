#!/bin/sh
# move2kube_amd detector: Maven build (pom.xml).
test -f "$1/pom.xml" || exit 1
printf '%s\n' '{"port": 8080, "app_name": "app"}'
