"""vboc_amd - MI355X-native batched boundary-OCP solver for VBOC data generation."""
