"""move2kube_amd - a from-scratch re-implementation of the move2kube migration
tool (collect / plan / translate of docker-compose, Cloud Foundry, Dockerfile,
source-directory and Kubernetes/Knative inputs into Kubernetes/Helm/Knative/
Tekton artifacts) with a native runtime: a C++ extension for directory
indexing, Dockerfile sniffing, hashing, batched edit distance and a parallel
detector-process pool, plus a gfx950 HIP kernel for large all-pairs fuzzy
matching.  See SURVEY.md for the component map.
"""

from .models.info import VERSION as __version__  # noqa: F401
