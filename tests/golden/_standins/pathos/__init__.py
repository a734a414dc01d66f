# Fixture-generation stand-in package for `pathos` (not installed).
