"""Command-line apps (reference src/ska_sdp_cip/apps/)."""
