"""Source translators: each turns one kind of input (directories, Dockerfiles, compose, CF manifests, k8s/knative YAMLs) into plan services and then IR."""
