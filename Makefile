# move2kube_amd developer entry points.
#   make build      native host extension + gfx950 HIP library (in-tree)
#   make test       CPU test suite (what CI runs)
#   make stress     race/stress harness (scripts/stress.py, 20 seeds)
#   make coverage   line coverage of the CPU suite (scripts/coverage.py)
#   make test-gpu   GPU tests (needs an MI355X)
#   make bench      headline benchmark (translate throughput on samples/)
#   make dist       sdist/wheel-style tarballs + sha256 sums under dist/
#   make cbuild     container image (cimage-e2e: translate samples/ inside it)
#   make installdeps  external tools (pack, kubectl, operator-sdk) into ./bin

PYTHON      ?= python3
IMAGE       ?= quay.io/konveyor/move2kube-amd
VERSION     ?= $(shell $(PYTHON) -c "from move2kube_amd.models.info import VERSION; print(VERSION)")
GIT_COMMIT  ?= $(shell git rev-parse HEAD 2>/dev/null)
GIT_DIRTY   ?= $(shell test -n "`git status --porcelain 2>/dev/null`" && echo dirty || echo clean)
OFFLOAD_ARCH ?= gfx950

.DEFAULT_GOAL := help

.PHONY: help
help: ## This help.
	@awk 'BEGIN {FS = ":.*?## "} /^[a-zA-Z0-9_-]+:.*?## / {printf "\033[36m%-14s\033[0m %s\n", $$1, $$2}' $(MAKEFILE_LIST)

.PHONY: build
build: ## Build the native extension and the HIP kernel library in-tree
	PYTORCH_ROCM_ARCH=$(OFFLOAD_ARCH) $(PYTHON) -m move2kube_amd.ops.build

.PHONY: generate
generate: ## Regenerate embedded asset modules
	$(PYTHON) -m move2kube_amd.utils.codegen move2kube_amd/assets/m2kassets maketar move2kube_amd/assets/_embedded_assets.py

.PHONY: test
test: build ## Run the CPU test suite
	$(PYTHON) -m pytest tests -q -m "not gpu"

.PHONY: stress
stress: build ## Race/stress harness: 20 seeded CLI runs per configuration under a 1 us switch interval
	$(PYTHON) scripts/stress.py --seeds 20

.PHONY: test-twins
test-twins: build ## Golden trees through every implementation twin (M2K_DISABLE_NATIVE=1 etc.)
	$(PYTHON) -m pytest tests/test_twin_matrix.py -q

.PHONY: test-gpu
test-gpu: build ## Run the GPU tests (MI355X)
	$(PYTHON) -m pytest tests -q -m gpu

.PHONY: test-coverage
test-coverage: build ## CPU tests with line coverage, checked against scripts/coverage_floor.json
	$(PYTHON) scripts/coverage.py run --floor scripts/coverage_floor.json

.PHONY: coverage
coverage: test-coverage

.PHONY: test-style
test-style: ## Syntax/byte-compile check and license-free header check
	$(PYTHON) -m compileall -q move2kube_amd tests bench.py __graft_entry__.py
	$(PYTHON) scripts/stylecheck.py

.PHONY: bench
bench: build ## Headline benchmark on 1 device
	$(PYTHON) bench.py --steps 20 --warmup 3

.PHONY: ci
ci: clean build test test-style ## Run the CI routine

.PHONY: dist
dist: clean build ## Build distribution archives + checksums
	$(PYTHON) scripts/builddist.py --version $(VERSION) --commit "$(GIT_COMMIT)" --tree "$(GIT_DIRTY)"

.PHONY: clean
clean: ## Remove build outputs (keeps the in-tree extensions)
	rm -rf dist build *.egg-info .pytest_cache

.PHONY: info
info: ## Version info
	@echo "Version:    $(VERSION)"
	@echo "Git Commit: $(GIT_COMMIT)"
	@echo "Git Tree:   $(GIT_DIRTY)"
	@echo "Arch:       $(OFFLOAD_ARCH)"

.PHONY: cbuild
cbuild: ## Build the container image
	docker build -t $(IMAGE):$(VERSION) --build-arg VERSION=$(VERSION) --build-arg GIT_COMMIT=$(GIT_COMMIT) \
		--build-arg GIT_TREE_STATE=$(GIT_DIRTY) .

.PHONY: cpush
cpush: ## Push the container image
	docker push $(IMAGE):$(VERSION)

.PHONY: cimage-e2e
cimage-e2e: ## Translate samples/ inside the built image and diff against the expected tree
	bash scripts/image_e2e.sh $(IMAGE):$(VERSION)

.PHONY: installdeps
installdeps: ## Install pack, kubectl and operator-sdk into ./bin (scripts/installdeps.sh)
	bash scripts/installdeps.sh
