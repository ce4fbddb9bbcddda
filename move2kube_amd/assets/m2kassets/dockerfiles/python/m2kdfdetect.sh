#!/bin/sh
# move2kube_amd detector: Python project (requirements.txt / setup.py /
# environment.yml / Pipfile).  POSIX sh: runs under dash as well as bash.
src="$1"
for marker in requirements.txt setup.py environment.yml Pipfile; do
    if [ -f "$src/$marker" ]; then
        main=$(grep -lRe "__main__" "$src" 2>/dev/null | awk '/.py$/ {print}' | head -n 1)
        rel=""
        [ -n "$main" ] && rel=$(realpath --relative-to="$src" "$main")
        printf '{"main_script_rel_path": "%s", "app_name": "app", "port": 8080}' "$rel"
        exit 0
    fi
done
exit 1
