#!/bin/sh
# move2kube_amd S2I detector: PHP (any *.php file).
n=$(find "$1"/. -name '*.php' -print 2>/dev/null | head -n 1 | wc -l)
[ "$n" -eq 1 ] || exit 1
printf '{"builder": "%s", "port": 8080}\n' "registry.access.redhat.com/rhscl/php-72-rhel7:latest"
