#!/bin/sh
# move2kube_amd detector: Ruby project (Gemfile).
test -f "$1/Gemfile" || exit 1
printf '%s\n' '{"port": 8080, "app_name": "app"}'
