"""Command-line entry points with the reference's flag names."""
