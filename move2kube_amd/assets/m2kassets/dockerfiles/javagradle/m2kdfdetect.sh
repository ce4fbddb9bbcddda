#!/bin/sh
# move2kube_amd detector: Gradle build (build.gradle).
test -f "$1/build.gradle" || exit 1
printf '%s\n' '{"port": 8080, "app_name": "simplewebapp"}'
