# Developer entry points (CI runs the same targets: .github/workflows/ci.yml).
PY ?= python3
ARCH ?= gfx950
JOBS ?= 8

.PHONY: all build build-san lint test test-gpu sanitize smoke bench bench-gemm image clean

all: build test

build:                      ## native libs: SMI library + CLI, HIP quota shim, DevicePlugin server, gfx950 kernels
	PYTORCH_ROCM_ARCH=$(ARCH) $(PY) native/build.py -j $(JOBS)
	$(PY) -c "import __graft_entry__ as g; g.build()"

build-san:                  ## host-side ASan+UBSan and TSan variants (_native/asan, _native/tsan)
	$(PY) native/build.py gpuinfo hipshim dpserver hbmbroker comgrcache --sanitize asan
	$(PY) native/build.py gpuinfo hipshim dpserver --sanitize tsan

lint:                       ## byte-compile everything; reject tabs / trailing whitespace in sources
	$(PY) -m compileall -q aliyun_gpushare_device_plugin_amd tests tools bench.py __graft_entry__.py
	! grep -rnP "\t|[ ]+$$" --include=*.py aliyun_gpushare_device_plugin_amd tests tools bench.py

test: build                 ## CPU suite (fake SMI, fake apiserver/kubelet, gloo multi-process)
	$(PY) -m pytest tests -q -m "not gpu"

sanitize: build-san         ## the sanitizer runs only
	$(PY) -m pytest tests -q -m "not gpu" -k "sanitizer or concurrent"

test-gpu: build             ## on an MI355X: kernels, shim on real HIP, plugin on real SMI
	$(PY) -m pytest tests -q -m gpu

smoke: build
	$(PY) -c "import __graft_entry__ as g; g.smoke()"

bench: build                ## 1-GPU headline bench (pods/s + Allocate latency under MFMA traffic)
	$(PY) bench.py --gpus 1

bench-gemm: build
	$(PY) tools/bench_gemm.py

image:                      ## deployable image (deploy/Dockerfile)
	docker build -f deploy/Dockerfile -t gpushare-device-plugin-mi355x:dev .

clean:
	rm -rf aliyun_gpushare_device_plugin_amd/_native .pytest_cache .hypothesis
