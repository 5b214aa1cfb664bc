"""MI355X-native multi-camera extrinsic bundle adjustment."""
