# Container recipe (reference: Dockerfile on a CUDA 11.8 base). ROCm + PyTorch-ROCm base;
# the HIP extension is cross-compiled for gfx950 (MI355X) at build time.
FROM rocm/pytorch:latest
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /workspace/imitation_amd
COPY . .
RUN pip install --no-cache-dir -e . && python -c "import __graft_entry__ as g; g.build()"
CMD ["python", "-m", "pytest", "tests", "-q", "-m", "not gpu"]
