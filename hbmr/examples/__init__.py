"""Example jobs (the reference's src/examples + src/examples/pipes, hbmr-native)."""
