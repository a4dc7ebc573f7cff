"""Stub `isaacgym` package used ONLY to import the reference's tensor code in the
build container and record golden vectors (tests/golden/). Never shipped, never
imported by the product path. See SURVEY.md Appendix D."""
