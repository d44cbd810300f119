# shared build settings of the image family (docker buildx; one platform: linux/amd64 — MI355X hosts)
REGISTRY ?= kfamd
TAG ?= $(shell git describe --tags --always --dirty 2>/dev/null || echo dev)
ROCM_VERSION ?= 7.0
GFX_ARCH ?= gfx950
BUILDX ?= docker buildx build --platform linux/amd64
BUILD_ARGS = --build-arg BASE_IMG_REGISTRY=$(REGISTRY) --build-arg BASE_IMG_TAG=$(TAG) \
             --build-arg ROCM_VERSION=$(ROCM_VERSION) --build-arg GFX_ARCH=$(GFX_ARCH)

define build_image
	$(BUILDX) $(BUILD_ARGS) -t $(REGISTRY)/$(1):$(TAG) -f $(2)/Dockerfile $(3) --load
endef
