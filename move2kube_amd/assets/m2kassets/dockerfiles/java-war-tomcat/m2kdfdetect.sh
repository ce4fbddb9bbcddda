#!/bin/sh
# move2kube_amd detector: prebuilt WAR file (deployed on tomcat).
for war in "$1"/*.war; do
    [ -e "$war" ] || exit 1
    count=$(ls -1 "$1"/*.war 2>/dev/null | wc -l)
    [ "$count" -gt 1 ] && echo "there are multiple WAR files. taking only the first one: $war" 1>&2
    printf '{"port":8080, "war_path":"%s"}' "$(basename "$war")"
    exit 0
done
exit 1
