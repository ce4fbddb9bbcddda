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
LABEL org.opencontainers.image.title="move2kube-amd" org.opencontainers.image.version="${VERSION}"
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-yaml python3-numpy git openssh-client \
 && rm -rf /var/lib/apt/lists/*
COPY --from=builder /src/move2kube_amd /opt/move2kube-amd/move2kube_amd
COPY --from=builder /src/samples /opt/move2kube-amd/samples
RUN printf '#!/bin/sh\nPYTHONPATH=/opt/move2kube-amd exec python3 -m move2kube_amd "$@"\n' > /usr/local/bin/move2kube \
 && chmod +x /usr/local/bin/move2kube
VOLUME /wksps
WORKDIR /wksps
ENTRYPOINT ["move2kube"]
CMD ["--help"]
