# pdo — MI355X-native PaddleJob operator + launcher
PY ?= python3
IMG_MANAGER ?= pdo/manager:rocm7.2
IMG_LAUNCHER ?= pdo/launcher:rocm7.2-torch2.10
GPURUN ?= /usr/local/graft/bin/gpurun

.PHONY: all build build-hip build-core clean test test-gpu test-core bench bench-launch manifests \
        manifests-check docker-build deploy undeploy sanitize license license-check

all: build

build:                 ## HIP kernels (gfx950) + native control plane + pybind modules
	$(PY) tools/build.py
build-hip:
	$(PY) tools/build.py --only hip
build-core:
	$(PY) tools/build.py --only core
clean:
	$(PY) tools/build.py --clean

test:                  ## CPU suite (control plane, launcher, gloo multi-process)
	$(PY) -m pytest tests -x -q -m "not gpu"
test-core: build-core  ## native C++ unit tests
	./bin/pdo-core-tests
test-gpu:              ## GPU numerics + workloads on an MI355X box
	$(GPURUN) --timeout 900 -- 'timeout -k 10 800 $(PY) -m pytest tests -m gpu -x -q'

bench:                 ## headline training throughput (1 GPU; torchrun for N>1)
	$(PY) bench.py
bench-launch:          ## job-start -> all-ranks-ready p50 (compat / fast / fast+zygote)
	$(PY) bench_launch.py --ranks 1 --trials 10

manifests:             ## regenerate deploy/ config/ charts/*/crds
	$(PY) -m paddle_operator_amd.deploy
manifests-check:
	$(PY) -m paddle_operator_amd.deploy --check

SAN_CMAKE = -G Ninja -DCMAKE_BUILD_TYPE=Debug -Dpybind11_DIR=$$($(PY) -c 'import pybind11;print(pybind11.get_cmake_dir())')
sanitize:              ## host-only ASan+UBSan and TSan builds of the control plane, run the native tests
	cmake -S csrc -B build/asan $(SAN_CMAKE) -DPDO_SANITIZE=address,undefined -DPDO_BIN_DIR=$(CURDIR)/build/asan/bin -DPDO_PKG_DIR=$(CURDIR)/build/asan/pkg
	ninja -C build/asan pdo-core-tests && UBSAN_OPTIONS=halt_on_error=1 build/asan/bin/pdo-core-tests
	cmake -S csrc -B build/tsan $(SAN_CMAKE) -DPDO_SANITIZE=thread -DPDO_BIN_DIR=$(CURDIR)/build/tsan/bin -DPDO_PKG_DIR=$(CURDIR)/build/tsan/pkg
	ninja -C build/tsan pdo-core-tests && TSAN_OPTIONS=halt_on_error=1 build/tsan/bin/pdo-core-tests

docker-build:
	docker build --target manager -t $(IMG_MANAGER) .
	docker build --target launcher -t $(IMG_LAUNCHER) .
deploy:
	kubectl apply -f deploy/v1/crd.yaml -f deploy/v1/operator.yaml
undeploy:
	kubectl delete -f deploy/v1/operator.yaml -f deploy/v1/crd.yaml

license:               ## add SPDX headers to sources that lack them
	$(PY) tools/license.py --fix
license-check:
	$(PY) tools/license.py
