from http.server import HTTPServer, SimpleHTTPRequestHandler

HTTPServer(("", 5000), SimpleHTTPRequestHandler).serve_forever()
