"""HIP backend: ctypes C-ABI binding (lib), recorded launch programs (program), network
builders (net), autograd Functions (autograd) and the static execution engine (engine)."""
