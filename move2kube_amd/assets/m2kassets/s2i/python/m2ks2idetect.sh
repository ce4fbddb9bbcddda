#!/bin/sh
# move2kube_amd S2I detector: Python (requirements.txt / setup.py /
# environment.yml / Pipfile).
src="$1"
for marker in requirements.txt setup.py environment.yml Pipfile; do
    if [ -f "$src/$marker" ]; then
        main=$(grep -lRe "__main__" "$src" 2>/dev/null | awk '/.py$/ {print}' | head -n 1)
        rel=""
        [ -n "$main" ] && rel=$(realpath --relative-to="$src" "$main")
        printf '{"builder": "%s", "app_file": "%s", "app_name": "app", "port": 8080}' \
            "registry.access.redhat.com/rhscl/python-36-rhel7:latest" "$rel"
        exit 0
    fi
done
exit 1
