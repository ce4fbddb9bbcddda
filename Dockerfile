# move2kube_amd container image (reference Dockerfile: a builder stage that
# runs scripts/installdeps.sh -y, then a runtime image with the CLI and
# operator-sdk).
#
# Builder: the ROCm toolchain compiles the native host extension (g++) and the
# gfx950 fuzzy-matching kernel library (hipcc), runs the CPU test suite, and
# installs operator-sdk, pack and kubectl with scripts/installdeps.sh.
# Runtime: a slim Python image - every command runs on the host CPUs.  The
# HIP library is only shipped with WITH_HIP=1 on a ROCm runtime base
#   docker build --build-arg RUNTIME_IMAGE=rocm/dev-ubuntu-22.04:7.2 --build-arg WITH_HIP=1 .
# (no move2kube command needs it; it serves the batched fuzzy matching API).
ARG ROCM_IMAGE=rocm/dev-ubuntu-22.04:7.2
ARG RUNTIME_IMAGE=python:3.10-slim-bookworm

FROM ${ROCM_IMAGE} AS builder
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip g++ make git curl ca-certificates libssl-dev \
 && python3 -m pip install --no-cache-dir pybind11 pyyaml numpy pytest hypothesis \
 && rm -rf /var/lib/apt/lists/*
WORKDIR /src
# external tools first (their own layer, reused while the sources change)
ARG OPERATOR_SDK_VERSION=v1.0.0
ARG OPERATOR_SDK_URL=
ARG PACK_VERSION=v0.12.0
ARG KUBECTL_VERSION=
COPY scripts/installdeps.sh scripts/installdeps.sh
# (the ARGs reach the script as environment variables; empty means its default).
# FORCE_INSTALL=1: all three tools land in /opt/m2k-deps even when the builder
# base already has one on PATH, so the runtime stage's COPY always finds them
RUN INSTALL_DOCKER=0 FORCE_INSTALL=1 MOVE2KUBE_DEP_INSTALL_PATH=/opt/m2k-deps bash scripts/installdeps.sh -y \
 && test -x /opt/m2k-deps/operator-sdk && test -x /opt/m2k-deps/pack && test -x /opt/m2k-deps/kubectl
COPY . .
RUN PYTORCH_ROCM_ARCH=gfx950 python3 -m move2kube_amd.ops.build \
 && python3 -m pytest tests -q -m "not gpu" -x -p no:cacheprovider

FROM ${RUNTIME_IMAGE}
ARG VERSION=latest
ARG GIT_COMMIT=""
ARG GIT_TREE_STATE=""
ARG WITH_HIP=0
LABEL org.opencontainers.image.title="move2kube-amd" org.opencontainers.image.version="${VERSION}"
RUN apt-get update && apt-get install -y --no-install-recommends git openssh-client \
 && rm -rf /var/lib/apt/lists/* \
 && (python3 -c "import yaml, numpy" 2>/dev/null || python3 -m pip install --no-cache-dir pyyaml numpy)
COPY --from=builder /opt/m2k-deps/operator-sdk /opt/m2k-deps/pack /opt/m2k-deps/kubectl /usr/local/bin/
COPY --from=builder /src/move2kube_amd /opt/move2kube-amd/move2kube_amd
COPY --from=builder /src/samples /opt/move2kube-amd/samples
# version stamp (the reference's -ldflags -X) and a launcher that runs the
# package by file, so a move2kube_amd directory in /wksps cannot shadow it; the
# start-up cache is rebuilt for this stage's interpreter (its compiled regexes
# are only used by the interpreter build that made them)
RUN printf 'VERSION = "%s"\nBUILD_METADATA = ""\nGIT_COMMIT = "%s"\nGIT_TREE_STATE = "%s"\n' \
      "${VERSION}" "${GIT_COMMIT}" "${GIT_TREE_STATE}" > /opt/move2kube-amd/move2kube_amd/_buildinfo.py \
 && if [ "${WITH_HIP}" != 1 ]; then rm -f /opt/move2kube-amd/move2kube_amd/ops/libm2k_ed_hip.so; fi \
 && printf 'import sys\nsys.path.insert(0, "/opt/move2kube-amd")\nfrom move2kube_amd.cli.main import main\nsys.exit(main())\n' \
      > /opt/move2kube-amd/m2k_main.py \
 && printf '#!/bin/sh\nexec python3 /opt/move2kube-amd/m2k_main.py "$@"\n' > /usr/local/bin/move2kube \
 && chmod +x /usr/local/bin/move2kube \
 && python3 -m compileall -q /opt/move2kube-amd/move2kube_amd \
 && (cd /opt/move2kube-amd && python3 -m move2kube_amd.ops.startcache_build >/dev/null) \
 && operator-sdk version && move2kube version
VOLUME /wksps
WORKDIR /wksps
ENTRYPOINT ["move2kube"]
CMD ["--help"]
