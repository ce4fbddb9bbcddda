#!/bin/sh
# move2kube_amd S2I detector: Ruby (Gemfile).
test -f "$1/Gemfile" || exit 1
printf '{"builder": "%s", "port": 8080}\n' "registry.access.redhat.com/rhscl/ruby-25-rhel7:latest"
