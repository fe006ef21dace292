"""``run_*`` entry points with the reference's flags."""
