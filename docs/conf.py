project = "p2pfl_amd"
extensions = ["myst_parser"]
source_suffix = {".md": "markdown"}
master_doc = "index"
html_theme = "alabaster"
