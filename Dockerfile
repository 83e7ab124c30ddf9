# MI355X image: ROCm PyTorch + the in-tree gfx950 extension.
#   docker build -t p2pfl-amd .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --ipc=host p2pfl-amd \
#       python bench.py --gpus 8 --steps 20 --warmup 5
# (the reference ships a CPU-torch image: /root/reference/Dockerfile)
FROM rocm/pytorch:latest
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /opt/p2pfl_amd
COPY . .
RUN pip install --no-cache-dir grpcio protobuf typer rich psutil safetensors msgpack pytest pytest-timeout \
 && python setup.py build_ext --inplace \
 && python -c "import __graft_entry__ as g; g.build()"
ENV PYTHONPATH=/opt/p2pfl_amd
CMD ["python", "-m", "p2pfl_amd", "--help"]
