"""FaceEnhanceNet on MI355X: the reference's `src` package surface (models, training) backed by
hand-written gfx950 HIP kernels (src/hip -> libfen_hip.so)."""
