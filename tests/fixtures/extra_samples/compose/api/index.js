require("http").createServer((q, r) => r.end("api\n")).listen(3000);
