require("http").createServer((q, r) => r.end("cf\n")).listen(process.env.PORT || 8080);
