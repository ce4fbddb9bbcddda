# move2kube_amd container image (reference Dockerfile: UBI8 builder -> runtime).
# Builder: compile the native host extension and the gfx950 kernel library with
# the ROCm toolchain.  Runtime: ROCm userspace + python; the GPU path is used
# when the container is started with /dev/kfd and /dev/dri passed through,
# everything else runs on the host CPUs.
ARG ROCM_IMAGE=rocm/dev-ubuntu-22.04:7.2
FROM ${ROCM_IMAGE} AS builder
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip g++ make git \
 && python3 -m pip install --no-cache-dir pybind11 pyyaml numpy \
 && rm -rf /var/lib/apt/lists/*
WORKDIR /src
COPY . .
RUN PYTORCH_ROCM_ARCH=gfx950 python3 -m move2kube_amd.ops.build \
 && python3 -m pytest tests -q -m "not gpu" -x

FROM ${ROCM_IMAGE}
ARG VERSION=latest
ARG GIT_COMMIT=""
ARG GIT_TREE_STATE=""
LABEL org.opencontainers.image.title="move2kube-amd" org.opencontainers.image.version="${VERSION}"
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-yaml python3-numpy git openssh-client \
 && rm -rf /var/lib/apt/lists/*
COPY --from=builder /src/move2kube_amd /opt/move2kube-amd/move2kube_amd
COPY --from=builder /src/samples /opt/move2kube-amd/samples
# version stamp (the reference's -ldflags -X) and a launcher that runs the
# package by file, so a move2kube_amd directory in /wksps cannot shadow it
RUN printf 'VERSION = "%s"\nBUILD_METADATA = ""\nGIT_COMMIT = "%s"\nGIT_TREE_STATE = "%s"\n' \
      "${VERSION}" "${GIT_COMMIT}" "${GIT_TREE_STATE}" > /opt/move2kube-amd/move2kube_amd/_buildinfo.py \
 && printf 'import sys\nsys.path.insert(0, "/opt/move2kube-amd")\nfrom move2kube_amd.cli.main import main\nsys.exit(main())\n' \
      > /opt/move2kube-amd/m2k_main.py \
 && printf '#!/bin/sh\nexec python3 /opt/move2kube-amd/m2k_main.py "$@"\n' > /usr/local/bin/move2kube \
 && chmod +x /usr/local/bin/move2kube \
 && python3 -m compileall -q /opt/move2kube-amd/move2kube_amd
VOLUME /wksps
WORKDIR /wksps
ENTRYPOINT ["move2kube"]
CMD ["--help"]
