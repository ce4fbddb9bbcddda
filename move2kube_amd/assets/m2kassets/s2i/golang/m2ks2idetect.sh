#!/bin/sh
# move2kube_amd S2I detector: Go (go.mod, or any *.go file).
src="$1"
builder="registry.access.redhat.com/ubi8/go-toolset:latest"
if [ ! -f "$src/go.mod" ]; then
    n=$(find "$src"/. -name '*.go' -print 2>/dev/null | head -n 1 | wc -l)
    [ "$n" -eq 1 ] || exit 1
fi
printf '{"builder": "%s", "port": 8080}\n' "$builder"
