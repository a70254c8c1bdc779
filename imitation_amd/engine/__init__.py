"""Device-resident training engines (whole rounds on the GPU)."""
