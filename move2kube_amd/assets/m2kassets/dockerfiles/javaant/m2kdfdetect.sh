#!/bin/sh
# move2kube_amd detector: Apache Ant build (build.xml).
test -f "$1/build.xml" || exit 1
printf '%s\n' '{"port": 8080, "ant_cmd": "ant all", "app_name": "simplewebapp"}'
